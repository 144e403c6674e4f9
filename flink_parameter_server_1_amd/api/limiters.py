"""Pull limiters: per-worker cap on in-flight pulls (the staleness bound).

* ``add_pull_limiter`` — buffering limiter (``M/WorkerLogic.scala:176-225``):
  at most ``pull_limit`` unanswered pulls; excess pull ids are queued FIFO and
  each answer releases one queued pull.
* ``add_blocking_pull_limiter`` — blocking limiter
  (``M/WorkerLogic.scala:82-156``): the pulling thread blocks on a condition
  until an answer arrives.  Only usable when pulls are issued from a thread
  other than the engine's worker loop (same restriction as the reference).
  Push/output are serialized under the same lock.

Both forward ``update_model`` so they also wrap worker logics with a
worker-resident model shard (``BaseMFWorkerLogic`` limiters,
``M/matrix/factorization/workers/BaseMFWorkerLogic.scala:39-187``).
"""
from __future__ import annotations

import threading
from collections import deque

from .logic import ParameterServerClient, WorkerLogic


class _LimitedClient(ParameterServerClient):
    def __init__(self, owner):
        self._owner = owner
        self.ps = None

    def pull(self, param_id):
        self._owner._limited_pull(param_id)

    def push(self, param_id, delta):
        self.ps.push(param_id, delta)

    def output(self, out):
        self.ps.output(out)


class PullLimitedWorkerLogic(WorkerLogic):
    """Buffering pull limiter decorator (see module docstring)."""

    def __init__(self, worker_logic: WorkerLogic, pull_limit: int):
        if pull_limit <= 0:
            raise ValueError("pull_limit must be positive")
        self.worker_logic = worker_logic
        self.pull_limit = pull_limit
        self.pull_counter = 0
        self.pull_queue = deque()
        self._client = _LimitedClient(self)

    def _limited_pull(self, param_id):
        if self.pull_counter < self.pull_limit:
            self.pull_counter += 1
            self._client.ps.pull(param_id)
        else:
            self.pull_queue.append(param_id)

    def open(self, ctx):
        self.worker_logic.open(ctx)

    def on_recv(self, data, ps):
        self._client.ps = ps
        self.worker_logic.on_recv(data, self._client)

    def on_pull_recv(self, param_id, value, ps):
        self._client.ps = ps
        self.worker_logic.on_pull_recv(param_id, value, self._client)
        self.pull_counter -= 1
        if self.pull_queue:
            self._limited_pull(self.pull_queue.popleft())

    def close(self):
        self.worker_logic.close()

    # worker-resident model forwarding (BaseMFWorkerLogic)
    def update_model(self, param_id, value):
        return self.worker_logic.update_model(param_id, value)

    @property
    def model(self):
        return self.worker_logic.model

    @property
    def pending_pulls(self) -> int:
        return self.pull_counter + len(self.pull_queue)


class _BlockingClient(ParameterServerClient):
    def __init__(self, owner):
        self._owner = owner
        self.ps = None

    def pull(self, param_id):
        o = self._owner
        with o._cond:
            while o.pull_counter >= o.pull_limit:
                o._cond.wait()
            o.pull_counter += 1
            self.ps.pull(param_id)

    def push(self, param_id, delta):
        with self._owner._cond:
            self.ps.push(param_id, delta)

    def output(self, out):
        with self._owner._cond:
            self.ps.output(out)


class BlockingPullLimitedWorkerLogic(WorkerLogic):
    """Blocking pull limiter decorator (see module docstring)."""

    def __init__(self, worker_logic: WorkerLogic, pull_limit: int):
        if pull_limit <= 0:
            raise ValueError("pull_limit must be positive")
        self.worker_logic = worker_logic
        self.pull_limit = pull_limit
        self.pull_counter = 0
        self._cond = None
        self._client = None
        self._ensure()

    def _ensure(self):
        if self._cond is None:
            self._cond = threading.Condition(threading.RLock())
            self._client = _BlockingClient(self)

    # locks are not copyable: recreate them in the copy (Flink would
    # serialize the logic per subtask the same way)
    def __deepcopy__(self, memo):
        import copy

        new = BlockingPullLimitedWorkerLogic.__new__(BlockingPullLimitedWorkerLogic)
        new.worker_logic = copy.deepcopy(self.worker_logic, memo)
        new.pull_limit = self.pull_limit
        new.pull_counter = 0
        new._cond = None
        new._client = None
        new._ensure()
        return new

    def _set_ps(self, ps):
        with self._cond:
            self._client.ps = ps

    def open(self, ctx):
        self.worker_logic.open(ctx)

    def on_recv(self, data, ps):
        self._set_ps(ps)
        self.worker_logic.on_recv(data, self._client)

    def on_pull_recv(self, param_id, value, ps):
        self._set_ps(ps)
        self.worker_logic.on_pull_recv(param_id, value, self._client)
        with self._cond:
            self.pull_counter -= 1
            self._cond.notify()

    def close(self):
        self.worker_logic.close()

    def update_model(self, param_id, value):
        return self.worker_logic.update_model(param_id, value)

    @property
    def model(self):
        return self.worker_logic.model


def add_pull_limiter(worker_logic: WorkerLogic, pull_limit: int) -> PullLimitedWorkerLogic:
    return PullLimitedWorkerLogic(worker_logic, pull_limit)


def add_blocking_pull_limiter(worker_logic: WorkerLogic, pull_limit: int) -> BlockingPullLimitedWorkerLogic:
    return BlockingPullLimitedWorkerLogic(worker_logic, pull_limit)


# Scala spelling
addPullLimiter = add_pull_limiter
addBlockingPullLimiter = add_blocking_pull_limiter
