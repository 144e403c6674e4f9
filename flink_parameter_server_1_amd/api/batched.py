"""Batched (tensor) worker API: the ``WorkerLogic`` contract over micro-batches.

The reference's worker is event-driven per record: ``onRecv(data, ps)`` issues
``ps.pull(id)``, ``onPullRecv(id, value, ps)`` issues ``ps.push(id, delta)`` and
``ps.output(out)`` (``M/WorkerLogic.scala:23-58``, ``M/ParameterServerClient.scala:12-20``).
The tensor engine (``core.tensor_engine``) runs the same contract on device
micro-batches:

``on_recv_batch(batch, ps)``
    one call per micro-batch; ``ps.pull(keys, payload)`` requests the
    parameters of ``keys`` (an int tensor, duplicates allowed).  ``payload`` is
    handed back with the answer (the reference keeps it in per-id FIFOs, e.g.
    ``ratingBuffer(item)``; here the answer is positional, so no queue is
    needed: answer row ``b`` belongs to request ``b``).
``on_pull_recv_batch(pulled, ps)``
    one call per ``pull``: ``pulled.values()`` are the ``[B, D]`` parameters in
    request order.  ``ps.push(deltas)`` pushes one delta row per request to the
    keys just answered (duplicates are pre-reduced on the worker: summed, or
    last-writer for ``set`` tables); ``ps.push_unique`` takes already reduced
    ``[U, D]`` rows (the fast path of fused kernels); ``ps.output(x)`` emits a
    worker output (``Left``).
``update_model_batch(ids, values)``
    worker-resident model load (``transformWithDoubleModelLoad``'s ``Right``
    records, ``M/FlinkParameterServer.scala:641-644``).
``on_eof(ps)``
    called once the whole input of every rank is consumed (the ``FlinkEOF``
    barrier).  It may return an iterable of further micro-batches, which go
    through ``on_recv_batch`` again -- how the offline (multi-epoch) MF worker
    replays its buffered ratings (``M/matrix/factorization/workers/PSOfflineMatrixFactorizationWorker.scala:96-127``).
    ``None`` ends the job.
``close(ps)``
    may emit final outputs.

Every call happens on the single owner thread of the rank (no foreign-thread
collector use).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Iterable, Optional

import torch

from .logic import RuntimeContext


@dataclass
class PulledBatch:
    """The answer to one ``pull``: unique rows + request -> row map."""

    keys: torch.Tensor        # [B] requested ids (as passed to pull)
    rows: torch.Tensor        # [U, D] one row per unique key (wire dtype)
    pos: torch.Tensor         # [B] int32: request b's row is rows[pos[b]]
    payload: Any = None
    #: under a locking PS logic only a subset of a pull is answered per round:
    #: positions of the answered requests within the original ``pull`` (else None)
    index: Optional[torch.Tensor] = None
    #: the pull was planned as the identity over the key space (``pos`` = the key)
    identity: bool = False

    def values(self) -> torch.Tensor:
        """``[B, D]`` parameter of every request, in request order (fp32; fp64
        when the rows travel as fp64, the bit-parity configuration)."""
        if self.rows.is_cuda and self.rows.dtype == torch.float32 and self.rows.dim() == 2:
            from .. import ops  # one native gather launch (the torch index took a cast + a gather)

            return ops.gather_rows(self.rows, self.pos)
        r = self.rows if self.rows.dtype == torch.float64 else self.rows.float()
        return r[self.pos.long()]

    @property
    def n_unique(self) -> int:
        return self.rows.shape[0]

    def __len__(self) -> int:
        return self.keys.numel()


class MaskedPair:
    """A ``(ids, values)`` output pair restricted to the rows where ``mask`` holds,
    compacted on first access.  Lets a worker emit a masked selection (e.g. the
    predictions of the unlabelled examples of a mixed micro-batch) without a host
    sync on the step: the consumer pays the compaction when it reads the output.
    Unpacks, indexes and iterates like the 2-tuple it stands for."""

    __slots__ = ("_ids", "_values", "_mask", "_pair")

    def __init__(self, ids: torch.Tensor, values: torch.Tensor, mask: torch.Tensor):
        self._ids, self._values, self._mask, self._pair = ids, values, mask, None

    def pair(self) -> tuple:
        if self._pair is None:
            self._pair = (self._ids[self._mask], self._values[self._mask])
            self._ids = self._values = self._mask = None
        return self._pair

    def __iter__(self):
        return iter(self.pair())

    def __getitem__(self, i):
        return self.pair()[i]

    def __len__(self) -> int:
        return 2

    def __repr__(self) -> str:
        return f"MaskedPair{self.pair()!r}"


class BatchedPSClient:
    """The worker's handle inside the tensor engine (see module docstring)."""

    def pull(self, keys: torch.Tensor, payload: Any = None) -> None:
        raise NotImplementedError

    def push(self, deltas: torch.Tensor, mask: Optional[torch.Tensor] = None) -> None:
        raise NotImplementedError

    def local_push_target(self, in_place: bool = False):
        """``(table, row_map)`` when the answered pull's push may be applied by the
        worker itself -- the owner is this rank (world 1), the PS rule is a plain
        additive one and the pulled rows are a snapshot, not the table -- else None.
        Adding the delta of pulled row ``r`` to ``table[row_map[r]]`` (float atomics)
        is then the push; call ``push_applied()`` afterwards instead of ``push*``.

        ``in_place=True``: the pulled rows may also BE the table (a zero-copy serve).
        The worker declares that it reads a row it has started updating only as
        "pulled row + what this micro-batch added so far" -- so updating the table row
        in place computes exactly what pushing the summed delta would (the MF tiled
        kernel's delta mode: a chunk continues from ``I + Dl``)."""
        return None

    def push_applied(self) -> None:
        """The answered pull's push was added to ``local_push_target()``'s table."""
        raise NotImplementedError

    def push_unique(self, deltas: torch.Tensor, mask: Optional[torch.Tensor] = None) -> None:
        raise NotImplementedError

    def push_keys(self, keys: torch.Tensor, deltas: torch.Tensor) -> None:
        raise NotImplementedError

    def output(self, out: Any) -> None:
        raise NotImplementedError


class BatchedWorkerLogic:
    """Subclass and override ``on_recv_batch`` / ``on_pull_recv_batch``.

    ``arbitrary_pushes = True`` declares that ``ps.push_keys`` may be used (to
    keys that were not pulled): the engine then runs one extra, collective
    planning round per micro-batch for them.  ``pushes = False`` declares a
    query-only worker (top-K serving): the engine skips the push round."""

    arbitrary_pushes = False
    pushes = True
    #: the callbacks are a pure device function of the batch and device state (no
    #: host syncs, no per-batch Python state, no buffer re-allocated after the first
    #: micro-batches of a shape): ``TensorRuntime(graph=True)`` may replay captured
    #: steps instead of calling them (``core.step_graph``)
    graph_safe = False

    def open(self, ctx: RuntimeContext) -> None:
        pass

    def on_recv_batch(self, batch: Any, ps: BatchedPSClient) -> None:
        raise NotImplementedError

    def on_pull_recv_batch(self, pulled: PulledBatch, ps: BatchedPSClient) -> None:
        raise NotImplementedError

    def update_model_batch(self, ids: torch.Tensor, values: torch.Tensor) -> None:
        raise NotImplementedError("this worker has no worker-resident model (double model load)")

    def on_eof(self, ps: BatchedPSClient) -> Optional[Iterable[Any]]:
        return None

    def close(self, ps: BatchedPSClient) -> None:
        pass


class FunctionBatchedWorkerLogic(BatchedWorkerLogic):
    """A batched worker from plain callables (tests / scripts)."""

    def __init__(self, on_recv_batch, on_pull_recv_batch, open=None, close=None,  # noqa: A002
                 graph_safe: bool = False):
        self._recv, self._answer, self._open, self._close = on_recv_batch, on_pull_recv_batch, open, close
        self.graph_safe = bool(graph_safe)

    def open(self, ctx):
        if self._open:
            self._open(ctx)

    def on_recv_batch(self, batch, ps):
        self._recv(batch, ps)

    def on_pull_recv_batch(self, pulled, ps):
        self._answer(pulled, ps)

    def close(self, ps):
        if self._close:
            self._close(ps)
