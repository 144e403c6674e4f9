"""Future-style worker API and the worker-resident-model worker base.

* ``WorkerLogicWithFuture`` / ``PSClientWithFuture`` / ``PullAnswerFuture``
  (``M/WorkerLogic.scala:239-356``): ``pull(id)`` returns a future completed
  by the per-id FIFO of waiters.  The reference's ``onComplete`` re-assigns
  its callback to a closure that calls itself (infinite recursion,
  ``M/WorkerLogic.scala:331-334``); here callbacks are kept in a
  list.  ``result()`` works when the answer has arrived (the reference throws
  unconditionally, ``:352-354``); blocking waits are supported when the
  engine runs the worker on another thread.
* ``BaseMFWorkerLogic`` (``M/matrix/factorization/workers/BaseMFWorkerLogic.scala:8-14``):
  a worker holding a worker-resident model shard, loaded by
  ``transform_with_double_model_load`` through ``update_model``.
"""
from __future__ import annotations

import threading
from collections import defaultdict, deque
from typing import Callable, Dict, List, Optional

from .logic import ParameterServerClient, WorkerLogic


class PullAnswerFuture:
    """Completed by the engine when the pull answer for ``param_id`` arrives."""

    def __init__(self, param_id: int):
        self.param_id = param_id
        self._callbacks: List[Callable] = []
        self._answer = None
        self._done = False
        self._event = threading.Event()

    def pull_arrived(self, param_id, param):
        self._answer = (param_id, param)
        self._done = True
        self._event.set()
        callbacks, self._callbacks = self._callbacks, []
        for cb in callbacks:
            cb(self._answer)

    def on_complete(self, f: Callable) -> None:
        if self._done:
            f(self._answer)
        else:
            self._callbacks.append(f)

    # Scala spelling
    onComplete = on_complete

    def is_completed(self) -> bool:
        return self._done

    isCompleted = is_completed

    @property
    def value(self):
        return self._answer if self._done else None

    def result(self, timeout: Optional[float] = None):
        if not self._event.wait(timeout):
            raise TimeoutError(f"pull answer for {self.param_id} did not arrive")
        return self._answer


class PSClientWithFuture:
    def pull(self, param_id: int) -> PullAnswerFuture:
        raise NotImplementedError

    def push(self, param_id: int, delta) -> None:
        raise NotImplementedError

    def output(self, out) -> None:
        raise NotImplementedError


class _FutureClient(PSClientWithFuture):
    def __init__(self, owner):
        self.owner = owner
        self.ps: Optional[ParameterServerClient] = None

    def pull(self, param_id):
        fut = PullAnswerFuture(param_id)
        self.owner._waiters[param_id].append(fut)
        self.ps.pull(param_id)
        return fut

    def push(self, param_id, delta):
        self.ps.push(param_id, delta)

    def output(self, out):
        self.ps.output(out)


class WorkerLogicWithFuture(WorkerLogic):
    """Subclass and implement ``on_data_recv(data, ps)`` (``ps.pull`` returns a future).

    Note: unlike the reference (``M/WorkerLogic.scala:264-269``), ``pull``
    actually sends the pull message to the PS (the reference only registers
    the waiter and never calls ``ps.pull``).
    """

    def __init__(self):
        self._waiters: Dict[int, deque] = defaultdict(deque)
        self._client = _FutureClient(self)

    def on_data_recv(self, data, ps: PSClientWithFuture) -> None:
        raise NotImplementedError

    onDataRecv = on_data_recv

    def on_recv(self, data, ps):
        self._client.ps = ps
        self.on_data_recv(data, self._client)

    def on_pull_recv(self, param_id, value, ps):
        self._client.ps = ps
        self._waiters[param_id].popleft().pull_arrived(param_id, value)


class BaseMFWorkerLogic(WorkerLogic):
    """Worker logic with a worker-resident model shard (``model: dict``)."""

    def __init__(self):
        self.model: Dict[int, object] = {}

    def update_model(self, param_id: int, value) -> None:
        self.model[param_id] = value

    updateModel = update_model
