"""Streaming micro-batch assembly for the tensor engine.

The reference decides message-batch boundaries with combinables
(``M/common/CombinationLogic.scala:12-33``): every message raises a
``CountLogic`` flag once ``max`` messages arrived (``M/common/CountLogic.scala:20-26``),
a ``TimerLogic`` thread raises its flag every ``interval`` if data arrived
(``M/common/TimerLogic.scala:13-26``), and a user predicate over the flags
(``AND`` / ``OR``, ``T/FlinkCombinationStackTest.scala:63-71``) flushes the buffer
and resets every flag.  Its timer flushes from a foreign thread.

``MicroBatcher`` applies the same policies to an unbounded record source, but
the decisions are taken on the single owner thread: a reader thread only feeds
a queue, the owner thread waits on it with a timeout equal to the next timer
tick, so a tick is handled exactly when it is due and no collector is ever
called from another thread.  Each flush yields ``collate(records)`` -- a device
micro-batch for ``core.tensor_engine``.  The source ends the stream, or
``idle_timeout_ms`` without a record does (``iterationWaitTime``,
``M/FlinkParameterServer.scala:49-52``): the buffered records are flushed
first.
"""
from __future__ import annotations

import queue
import threading
import time
from typing import Any, Callable, Iterable, Iterator, List, Optional, Sequence

_END = object()


class FlushPolicy:
    """One combinable: a flag raised by records and / or clock ticks."""

    def __init__(self):
        self.flag = False

    def on_record(self) -> None:
        pass

    def next_tick(self) -> Optional[float]:
        return None

    def on_tick(self, now: float) -> None:
        pass

    def reset(self) -> None:
        self.flag = False


class CountPolicy(FlushPolicy):
    """Flag after every ``n`` records (the counter restarts when it fires)."""

    def __init__(self, n: int):
        super().__init__()
        if n <= 0:
            raise ValueError("count must be > 0")
        self.n, self.count = int(n), 0

    def on_record(self):
        self.count += 1
        if self.count >= self.n:
            self.flag = True
            self.count = 0


class TimerPolicy(FlushPolicy):
    """Flag at every tick (every ``interval_ms``, from the first record) at which
    records arrived since the previous tick."""

    def __init__(self, interval_ms: float, clock: Callable[[], float] = time.monotonic):
        super().__init__()
        if interval_ms <= 0:
            raise ValueError("interval must be > 0")
        self.interval = float(interval_ms) / 1000.0
        self.clock = clock
        self.contains_data = False
        self._next: Optional[float] = None

    def on_record(self):
        self.contains_data = True
        if self._next is None:
            self._next = self.clock() + self.interval

    def next_tick(self):
        return self._next

    def on_tick(self, now):
        if self._next is None or now < self._next:
            return
        while self._next <= now:
            self._next += self.interval
        if self.contains_data:
            self.flag = True
            self.contains_data = False


def all_of(policies: Sequence[FlushPolicy]) -> bool:
    return all(p.flag for p in policies)


def any_of(policies: Sequence[FlushPolicy]) -> bool:
    return any(p.flag for p in policies)


class MicroBatcher:
    """Iterate ``collate(records)`` micro-batches of an unbounded ``source``.

    ``policies`` + ``predicate`` (default: one policy, its flag) decide the flushes;
    ``max_records`` is a hard cap on a buffered batch (device memory), flushing
    regardless of the predicate."""

    def __init__(self, source: Iterable, policies: Sequence[FlushPolicy], predicate: Callable = any_of,
                 collate: Optional[Callable[[List[Any]], Any]] = None, idle_timeout_ms: Optional[float] = None,
                 max_records: Optional[int] = None, clock: Callable[[], float] = time.monotonic):
        self.source = source
        self.policies = list(policies)
        self.predicate = predicate
        self.collate = collate or (lambda recs: recs)
        self.idle = None if not idle_timeout_ms else float(idle_timeout_ms) / 1000.0
        self.max_records = max_records
        self.clock = clock
        self.flushes: List[int] = []  # sizes of the emitted batches (observability / tests)
        self.ended_by = None          # "source" | "idle"

    def _reader(self, q):
        try:
            for x in self.source:
                q.put(x)
        finally:
            q.put(_END)

    def __iter__(self) -> Iterator[Any]:
        q: "queue.Queue" = queue.Queue(maxsize=1 << 16)
        threading.Thread(target=self._reader, args=(q,), daemon=True).start()
        buf: List[Any] = []
        last_rec = self.clock()

        def flush():
            nonlocal buf
            out, buf = buf, []
            for p in self.policies:
                p.reset()
            self.flushes.append(len(out))
            return self.collate(out)

        while True:
            now = self.clock()
            ticks = [t for t in (p.next_tick() for p in self.policies) if t is not None]
            deadline = min(ticks) if ticks else None
            if self.idle is not None:
                idle_at = last_rec + self.idle
                deadline = idle_at if deadline is None else min(deadline, idle_at)
            wait = None if deadline is None else max(0.0, deadline - now)
            try:
                x = q.get(timeout=wait)
            except queue.Empty:
                x = None
                now = self.clock()
                for p in self.policies:
                    p.on_tick(now)
                if buf and self.predicate(self.policies):
                    yield flush()
                if self.idle is not None and now - last_rec >= self.idle:
                    self.ended_by = "idle"
                    if buf:
                        yield flush()
                    return
                continue
            if x is _END:
                self.ended_by = "source"
                if buf:
                    yield flush()
                return
            # ticks fall due whatever the record rate (``TimerLogic`` fires every
            # interval, ``M/common/TimerLogic.scala:13-26``): a saturated queue never
            # reaches the ``Empty`` branch above, so due ticks are handled here too
            now = self.clock()
            for p in self.policies:
                p.on_tick(now)
            buf.append(x)
            last_rec = now
            for p in self.policies:
                p.on_record()
            if self.predicate(self.policies) or (self.max_records and len(buf) >= self.max_records):
                yield flush()
