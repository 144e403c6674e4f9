"""Bounded-staleness pull/compute/push pipeline over a ``TensorPS``.

The reference bounds asynchrony per worker with ``pullLimit``: at most that many
pulls may be outstanding, later ones are queued (``M/WorkerLogic.scala:176-225``,
``PullLimitedWorkerLogic``).  Over micro-batches the same knob becomes a
*staleness bound*: with ``staleness = s`` the pull of micro-batch ``k`` is served
before the pushes of micro-batches ``k-s .. k-1`` are applied, never earlier ones.

* ``s = 0``: synchronous (pull k, compute k, push k);
* ``s = 1``: the row all-to-all of batch ``k+1`` runs while batch ``k`` computes
  (what ``models.mf.fast`` does);
* ``s > 1``: deeper pipelines for slow links / large tables (config #5 stress).

Everything is stream-ordered on the device, so the bound is exact: the gather of
batch ``k`` is enqueued after the apply of batch ``k-s-1``.
"""
from __future__ import annotations

from collections import deque
from typing import Any, Callable, List, Optional, Tuple

import torch

from .tensor_ps import PullPlan, TensorPS

#: compute(rows, plan, payload) -> (deltas [U, D] or None, result)
ComputeFn = Callable[[torch.Tensor, PullPlan, Any], Tuple[Optional[torch.Tensor], Any]]


class BoundedStalenessPipeline:
    def __init__(self, ps: TensorPS, compute: ComputeFn, staleness: int = 1, lr: float = 0.0):
        if staleness < 0:
            raise ValueError("staleness must be >= 0")
        self.ps, self.compute, self.staleness, self.lr = ps, compute, int(staleness), lr
        self._q: deque = deque()
        self.max_observed = 0  # pushes of earlier batches still pending when a pull was served

    def submit(self, keys: torch.Tensor, payload: Any = None) -> List[Any]:
        """Issue the pull of a new micro-batch; finish (compute + push) every
        batch that would otherwise exceed the staleness bound.  Returns the
        results of the batches finished by this call, oldest first."""
        rows, work, plan = self.ps.pull_async(keys)
        self.max_observed = max(self.max_observed, len(self._q))
        self._q.append((rows, work, plan, payload))
        out = []
        while len(self._q) > self.staleness:
            out.append(self._finish(self._q.popleft()))
        return out

    def drain(self) -> List[Any]:
        out = []
        while self._q:
            out.append(self._finish(self._q.popleft()))
        return out

    @property
    def in_flight(self) -> int:
        return len(self._q)

    def _finish(self, item) -> Any:
        rows, work, plan, payload = item
        if work is not None:
            work.wait()
        deltas, result = self.compute(rows, plan, payload)
        if deltas is not None:
            self.ps.push(plan, deltas, lr=self.lr)
        return result
