"""L5 PS-side logic library (per-record compat path).

* ``SimplePSLogic`` — dict store, lazy init on first pull, push =
  ``update(old, delta)`` or ``delta`` if absent, emits ``(id, new)`` on every
  push (``M/server/SimplePSLogic.scala:7-26``).
* ``SimplePSLogicWithClose`` — same store, no per-push output, dumps the shard
  at close (``M/server/SimplePSLogicWithClose.scala:7-32``).
* ``RangePSLogicWithClose`` — dense shard for contiguous range partitioning
  (``M/server/RangePSLogicWithClose.scala:7-62``); ``div = ceil(F/P)``, last
  shard gets the remainder.  The reference's debug ``println`` is dropped
  (SURVEY B9).
* ``LockPSLogicA`` / ``LockPSLogicB`` — per-key read-modify-write locks: a
  pull locks the key until the matching push; other pullers queue (B: a
  worker index is queued at most once) (``M/server/LockPSLogicA.scala:13-46``,
  ``M/server/LockPSLogicB.scala:15-50``).

Every logic is also describable to the GPU path (``device_spec``) so the
tensor engine can run the same semantics as HBM-resident tables with fused
gather/apply kernels instead of a Python callback per key.
"""
from __future__ import annotations

import math
from collections import deque
from typing import Callable, Dict, List, Optional, Tuple

from ..api.logic import ParameterServer, ParameterServerLogic, RuntimeContext


class SimplePSLogic(ParameterServerLogic):
    def __init__(self, param_init: Callable[[int], object], param_update: Callable[[object, object], object]):
        self.init = param_init
        self.update = param_update
        self.params: Dict[int, object] = {}

    def on_pull_recv(self, param_id, worker_partition_index, ps: ParameterServer):
        params = self.params
        if param_id in params:
            v = params[param_id]
        else:
            v = params[param_id] = self.init(param_id)
        ps.answer_pull(param_id, v, worker_partition_index)

    def _apply(self, param_id, delta):
        params = self.params
        c = self.update(params[param_id], delta) if param_id in params else delta
        self.params[param_id] = c
        return c

    def on_push_recv(self, param_id, delta, ps: ParameterServer):
        c = self._apply(param_id, delta)
        ps.output((param_id, c))

    def device_spec(self):
        return {"kind": "simple", "emit_on_push": True}


class SimplePSLogicWithClose(SimplePSLogic):
    def on_push_recv(self, param_id, delta, ps: ParameterServer):
        self._apply(param_id, delta)

    def close(self, ps: ParameterServer):
        for k, v in self.params.items():
            ps.output((k, v))

    def device_spec(self):
        return {"kind": "simple", "emit_on_push": False}


def range_shard_bounds(feature_count: int, n_subtasks: int, subtask: int) -> Tuple[int, int]:
    """(start, size) of a range shard, exactly as ``RangePSLogicWithClose.open``."""
    div = int(math.ceil(feature_count / n_subtasks))
    mod = feature_count - (n_subtasks - 1) * div
    if mod != 0 and subtask + 1 == n_subtasks:
        size = mod
    else:
        size = div
    return subtask * div, max(size, 0)


class RangePSLogicWithClose(ParameterServerLogic):
    def __init__(self, feature_count: int, param_init, param_update):
        self.feature_count = feature_count
        self.init = param_init
        self.update = param_update
        self.start_index = 0
        self.params: List[Optional[object]] = []

    def open(self, config, ctx: RuntimeContext):
        self.start_index, size = range_shard_bounds(
            self.feature_count, ctx.number_of_parallel_subtasks, ctx.index_of_this_subtask
        )
        self.params = [None] * size

    def _local(self, param_id):
        idx = param_id - self.start_index
        if idx < 0 or idx >= len(self.params):
            raise IndexError(
                f"param {param_id} outside range shard [{self.start_index}, {self.start_index + len(self.params)})"
            )
        return idx

    def on_pull_recv(self, param_id, worker_partition_index, ps):
        idx = self._local(param_id)
        v = self.params[idx]
        if v is None:
            v = self.init(param_id)
            self.params[idx] = v
        ps.answer_pull(param_id, v, worker_partition_index)

    def on_push_recv(self, param_id, delta, ps):
        idx = self._local(param_id)
        old = self.params[idx]
        self.params[idx] = delta if old is None else self.update(old, delta)

    def close(self, ps):
        for i, v in enumerate(self.params):
            if v is not None:
                ps.output((self.start_index + i, v))

    def device_spec(self):
        return {"kind": "range", "feature_count": self.feature_count, "emit_on_push": False}


class LockPSLogicA(ParameterServerLogic):
    """``params[id] = [locked, value, queue]`` (list so tests can index like the tuple)."""

    dedup_queue = False

    def __init__(self, param_init, param_update):
        self.init = param_init
        self.update = param_update
        self.params: Dict[int, tuple] = {}

    def on_pull_recv(self, param_id, worker_partition_index, ps):
        entry = self.params.get(param_id)
        if entry is None:
            entry = (False, self.init(param_id), deque())
            self.params[param_id] = entry
        locked, p, q = entry
        if not locked:
            ps.answer_pull(param_id, p, worker_partition_index)
            self.params[param_id] = (True, p, q)
        else:
            if not (self.dedup_queue and worker_partition_index in q):
                q.append(worker_partition_index)

    def on_push_recv(self, param_id, delta, ps):
        entry = self.params.get(param_id)
        if entry is None:
            raise IllegalStateException("Not existed model was not able to update by any delta.")
        _, param, q = entry
        c = self.update(param, delta)
        if not q:
            self.params[param_id] = (False, c, q)
        else:
            ps.answer_pull(param_id, c, q.popleft())
            self.params[param_id] = (True, c, q)
        ps.output((param_id, c))

    def device_spec(self):
        return {"kind": "lock", "dedup_queue": self.dedup_queue, "emit_on_push": True}


class LockPSLogicB(LockPSLogicA):
    dedup_queue = True


class IllegalStateException(RuntimeError):
    """Same name as the JVM exception the reference throws."""
