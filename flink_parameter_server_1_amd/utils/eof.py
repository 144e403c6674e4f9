"""End-of-input detection for finite streams (``M/utils/FlinkEOF.scala:18-122``).

``flat_map_with_eof(sources, fn, parallelism, partitioner, key_selector)``:
every upstream source (one per element of ``sources``, run concurrently on
its own thread, like Flink source subtasks) routes its records to a
downstream subtask by ``partitioner(key_selector(x), parallelism)``; when a
source finishes it broadcasts ``EOF(src, tgt)`` to every downstream subtask
(``:97-107``).  A downstream subtask calls ``fn.on_eof(collect)`` once it
has counted one EOF per source (``:30-36``) -- a barrier: every record of
every source is processed before any ``on_eof``.  An empty source raises,
as the reference does (``:103-105``).

``fn`` is an object with ``flat_map(value, collect)`` and
``on_eof(collect)`` (optionally ``open(ctx)``); one copy per downstream
subtask.  Returns the per-subtask output lists.

``with_eof(data, parallelism, partitioner)`` is the engine-facing form: the
input split per worker with ``Left(EOF())`` appended to every partition
(what ``psOfflineMF`` feeds its workers, ``M/matrix/factorization/PSOfflineMatrixFactorization.scala:60-75``).
"""
from __future__ import annotations

import copy
import queue
import threading
import time
from typing import Callable, Iterable, List, Optional, Sequence

from ..api.logic import RuntimeContext
from ..core.engine import PartitionedInput, split_input
from ..core.messages import Left, Right


class EOF:
    """End-of-input marker (``case class EOF()``)."""

    def __eq__(self, other):
        return isinstance(other, EOF)

    def __hash__(self):
        return 0xE0F

    def __repr__(self):
        return "EOF()"


class EOFHandler:
    def on_eof(self, collect: Callable) -> None:
        raise NotImplementedError


class _EOFSignal:
    __slots__ = ("src", "tgt")

    def __init__(self, src, tgt):
        self.src, self.tgt = src, tgt


class IllegalStateException(RuntimeError):
    pass


def flat_map_with_eof(sources: Sequence[Iterable], fn, parallelism: int,
                      partitioner: Optional[Callable[[object, int], int]] = None,
                      key_selector: Callable = lambda x: x, timeout: float = 600.0) -> List[list]:
    n_src = len(sources)
    partitioner = partitioner or (lambda k, n: hash(k) % n)
    inboxes = [queue.Queue() for _ in range(parallelism)]
    errors: List[BaseException] = []

    def run_source(i, src):
        try:
            cnt = 0
            for x in src:
                inboxes[partitioner(key_selector(x), parallelism) % parallelism].put(x)
                cnt += 1
            if cnt == 0:
                raise IllegalStateException("Source subtask produced no record: EOF cannot be signalled.")
        except BaseException as e:  # noqa: BLE001
            errors.append(e)
        finally:
            for t in range(parallelism):
                inboxes[t].put(_EOFSignal(i, t))

    outputs: List[list] = [[] for _ in range(parallelism)]

    def run_sink(t):
        f = copy.deepcopy(fn)
        if hasattr(f, "open"):
            f.open(RuntimeContext(t, parallelism))
        seen = 0
        out = outputs[t].append
        try:
            while seen < n_src:
                x = inboxes[t].get(timeout=timeout)
                if isinstance(x, _EOFSignal):
                    seen += 1
                    continue
                f.flat_map(x, out)
            f.on_eof(out)
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=run_source, args=(i, s), daemon=True) for i, s in enumerate(sources)]
    threads += [threading.Thread(target=run_sink, args=(t,), daemon=True) for t in range(parallelism)]
    for th in threads:
        th.start()
    deadline = time.monotonic() + timeout  # one overall deadline, not one per thread
    for th in threads:
        th.join(max(0.0, deadline - time.monotonic()))
    if errors:
        raise errors[0]
    alive = [th.name for th in threads if th.is_alive()]
    if alive:  # a sink still waiting for EOFs: never hand back partial outputs
        raise TimeoutError(f"flat_map_with_eof: {len(alive)} subtask(s) did not finish within {timeout} s")
    return outputs


def with_eof(data, parallelism: int, partitioner: Optional[Callable] = None) -> PartitionedInput:
    """Split ``data`` over workers as ``Right(x)`` records, each partition ending in ``Left(EOF())``."""
    parts = split_input(data, parallelism, partitioner)
    return PartitionedInput([[Right(x) for x in p] + [Left(EOF())] for p in parts])


# Scala spelling
flatMapWithEOF = flat_map_with_eof
