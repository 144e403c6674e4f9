"""L4 user-facing API: worker logic, PS logic and their handles.

Same contract as the reference:

* ``WorkerLogic`` — ``open(ctx)``, ``on_recv(data, ps)``,
  ``on_pull_recv(param_id, value, ps)``, ``close()``
  (``M/WorkerLogic.scala:23-58``).
* ``ParameterServerClient`` — ``pull(id)``, ``push(id, delta)``,
  ``output(out)`` (``M/ParameterServerClient.scala:12-20``).
* ``ParameterServerLogic`` — ``on_pull_recv(id, worker_idx, ps)``,
  ``on_push_recv(id, delta, ps)``, ``close(ps)``, ``open(config, ctx)``
  (``M/FlinkParameterServer.scala:891-926``).
* ``ParameterServer`` — ``answer_pull(id, value, worker_idx)``,
  ``output(out)`` (``M/FlinkParameterServer.scala:928-932``).

camelCase aliases (``onRecv``, ``onPullRecv``, ``answerPull`` ...) are
provided so code written against the Scala API reads the same.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Generic, Optional, TypeVar

T = TypeVar("T")
P = TypeVar("P")
WOut = TypeVar("WOut")
PSOut = TypeVar("PSOut")


@dataclass
class RuntimeContext:
    """What Flink's ``RuntimeContext`` gives a subtask.

    ``index_of_this_subtask`` / ``number_of_parallel_subtasks`` are the
    values the reference reads (e.g. ``M/server/RangePSLogicWithClose.scala:51-62``).
    ``rank``/``world_size`` are the process-level coordinates when running
    one process per GPU; ``device`` is the torch device of the rank.
    """

    index_of_this_subtask: int = 0
    number_of_parallel_subtasks: int = 1
    rank: int = 0
    world_size: int = 1
    device: Any = "cpu"
    task_name: str = ""
    config: Dict[str, Any] = field(default_factory=dict)
    #: the rank's communicator (``parallel.comm.Comm`` or a virtual world's), for workers
    #: that exchange data of their own (the top-K workers' candidate gather)
    comm: Any = None

    # Flink-style accessors
    def getIndexOfThisSubtask(self) -> int:  # noqa: N802
        return self.index_of_this_subtask

    def getNumberOfParallelSubtasks(self) -> int:  # noqa: N802
        return self.number_of_parallel_subtasks


class ParameterServerClient(Generic[P, WOut]):
    """Worker's handle to the PS (fire-and-forget pull, delta push, output)."""

    def pull(self, param_id: int) -> None:
        raise NotImplementedError

    def push(self, param_id: int, delta: P) -> None:
        raise NotImplementedError

    def output(self, out: WOut) -> None:
        raise NotImplementedError


class ParameterServer(Generic[P, PSOut]):
    """PS shard's handle: answer a pull to a given worker, emit PS output."""

    def answer_pull(self, param_id: int, value: P, worker_partition_index: int) -> None:
        raise NotImplementedError

    def output(self, out: PSOut) -> None:
        raise NotImplementedError

    # Scala spelling
    def answerPull(self, param_id, value, worker_partition_index):  # noqa: N802
        return self.answer_pull(param_id, value, worker_partition_index)


class WorkerLogic(Generic[T, P, WOut]):
    """Event-driven worker: one callback per record and per pull answer."""

    def open(self, ctx: RuntimeContext) -> None:
        pass

    def on_recv(self, data: T, ps: ParameterServerClient) -> None:
        # Scala-named subclasses override onRecv instead.
        if type(self).onRecv is not WorkerLogic.onRecv:
            return self.onRecv(data, ps)
        raise NotImplementedError

    def on_pull_recv(self, param_id: int, value: P, ps: ParameterServerClient) -> None:
        if type(self).onPullRecv is not WorkerLogic.onPullRecv:
            return self.onPullRecv(param_id, value, ps)
        raise NotImplementedError

    def close(self) -> None:
        pass

    # Scala spelling (overridable)
    def onRecv(self, data, ps):  # noqa: N802
        return self.on_recv(data, ps)

    def onPullRecv(self, param_id, value, ps):  # noqa: N802
        return self.on_pull_recv(param_id, value, ps)


class ParameterServerLogic(Generic[P, PSOut]):
    """PS shard callbacks.  ``close`` may emit the final model."""

    def open(self, config: Optional[dict], ctx: RuntimeContext) -> None:
        pass

    def on_pull_recv(self, param_id: int, worker_partition_index: int, ps: ParameterServer) -> None:
        if type(self).onPullRecv is not ParameterServerLogic.onPullRecv:
            return self.onPullRecv(param_id, worker_partition_index, ps)
        raise NotImplementedError

    def on_push_recv(self, param_id: int, delta: P, ps: ParameterServer) -> None:
        if type(self).onPushRecv is not ParameterServerLogic.onPushRecv:
            return self.onPushRecv(param_id, delta, ps)
        raise NotImplementedError

    def close(self, ps: ParameterServer) -> None:
        pass

    def onPullRecv(self, param_id, worker_partition_index, ps):  # noqa: N802
        return self.on_pull_recv(param_id, worker_partition_index, ps)

    def onPushRecv(self, param_id, delta, ps):  # noqa: N802
        return self.on_push_recv(param_id, delta, ps)


class FunctionWorkerLogic(WorkerLogic):
    """Build a WorkerLogic from plain callables (handy for tests/scripts)."""

    def __init__(self, on_recv, on_pull_recv, open=None, close=None):  # noqa: A002
        self._on_recv = on_recv
        self._on_pull_recv = on_pull_recv
        self._open = open
        self._close = close

    def open(self, ctx):
        if self._open:
            self._open(ctx)

    def on_recv(self, data, ps):
        self._on_recv(data, ps)

    def on_pull_recv(self, param_id, value, ps):
        self._on_pull_recv(param_id, value, ps)

    def close(self):
        if self._close:
            self._close()
