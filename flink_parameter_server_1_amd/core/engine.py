"""L3 engine for the per-record (compat) path: ``transform`` and model load.

The reference builds a Flink streaming iteration: a worker ``CoFlatMap``
(training data + pull answers) -> custom-partitioned shuffle -> PS
``FlatMap`` -> custom-partitioned feedback edge back to the workers
(``M/FlinkParameterServer.scala:195-336``).  Outputs of both sides are
unioned as ``Either[WOut, PSOut]`` (``:319-328``).  Termination is an idle
timeout (``iterationWaitTime``, ``:49-52``).

Here there is no cyclic dataflow graph.  Each worker / PS subtask is a
mailbox with FIFO channels and a single owner loop drives them:

* ``LocalRuntime`` — all subtasks of a job in one process, one driver thread
  (deterministic scheduling, per-(sender, receiver) FIFO preserved, the
  property the MF workers rely on).
* ``DistRuntime`` (``core/dist_engine.py``) — one process per rank; the
  same subtasks exchange their outboxes in rounds over ``torch.distributed``
  (gloo on CPU, the Flink-mini-cluster analogue of the reference tests).

Termination is *global quiescence* (no queued message, no buffered
combination message, input exhausted) instead of an idle timeout; an
optional ``iteration_wait_time`` (ms) keeps the job alive that long after
quiescence for work injected by user threads (blocking limiter, timers).

The GPU fast path (``parallel/``) implements the same pull/push protocol
on tensors with RCCL all-to-all; this engine is the semantic reference the
parity tests compare it with.
"""
from __future__ import annotations

import copy
import itertools
import time
from collections import deque
from typing import Any, Callable, Iterable, List, Optional, Sequence

from ..api.logic import ParameterServer, ParameterServerClient, ParameterServerLogic, RuntimeContext, WorkerLogic
from ..ps.logics import SimplePSLogic
from ..utils.logs import message_tracing, trace_message
from .adapters import SimplePSReceiver, SimplePSSender, SimpleWorkerReceiver, SimpleWorkerSender
from .messages import Left, PSToWorker, Right, WorkerToPS
from .partitioners import hash_partition


# ---------------------------------------------------------------------------
# handles bound to a subtask (MessagingPSClient / MessagingPS analogues,
# M/FlinkParameterServer.scala:821-873).  They never swap collectors, so they
# are safe to call from user threads.
class _WorkerClient(ParameterServerClient):
    __slots__ = ("task", "engine")

    def __init__(self, task, engine):
        self.task = task
        self.engine = engine

    def pull(self, param_id):
        self.task.sender.on_pull(param_id, self.task.emit_to_ps, self.task.index)

    def push(self, param_id, delta):
        self.task.sender.on_push(param_id, delta, self.task.emit_to_ps, self.task.index)

    def output(self, out):
        self.engine.emit_output(Left(out))


class _PSHandle(ParameterServer):
    __slots__ = ("task", "engine")

    def __init__(self, task, engine):
        self.task = task
        self.engine = engine

    def answer_pull(self, param_id, value, worker_partition_index):
        self.task.sender.on_pull_answer(param_id, value, worker_partition_index, self.task.emit_to_worker)

    def output(self, out):
        self.engine.emit_output(Right(out))


class WorkerTask:
    def __init__(self, index, logic, sender, receiver, engine):
        self.index = index
        self.logic = logic
        self.sender = sender
        self.receiver = receiver
        self.engine = engine
        self.data = None  # iterator over this subtask's input partition
        self.answers = deque()
        self.client = _WorkerClient(self, engine)
        self.data_done = False
        self._on_answer = None

    def emit_to_ps(self, msg):
        self.engine.route_to_ps(msg)

    def handle_answer(self, wire_msg):
        if message_tracing():  # M/FlinkParameterServer.scala:247 (debug per pull answer)
            trace_message("worker <- ps", self.index, wire_msg)
        if self._on_answer is None:
            logic, client = self.logic, self.client
            self._on_answer = lambda pa: logic.on_pull_recv(pa.param_id, pa.param, client)
        self.receiver.on_pull_answer_recv(wire_msg, self._on_answer)

    def handle_data(self, rec):
        if message_tracing():  # M/FlinkParameterServer.scala:237 (debug per data record)
            trace_message("worker <- data", self.index, rec)
        self.logic.on_recv(rec, self.client)


class PSTask:
    def __init__(self, index, logic, sender, receiver, engine):
        self.index = index
        self.logic = logic
        self.sender = sender
        self.receiver = receiver
        self.engine = engine
        self.inbox = deque()
        self.handle = _PSHandle(self, engine)
        logic_, h = logic, self.handle
        self._on_pull = lambda pid, widx: logic_.on_pull_recv(pid, widx, h)
        self._on_push = lambda pid, delta: logic_.on_push_recv(pid, delta, h)

    def emit_to_worker(self, msg):
        self.engine.route_to_worker(msg)

    def handle_msg(self, wire_msg):
        if message_tracing():  # M/FlinkParameterServer.scala:284 (debug per PS message)
            trace_message("ps <- worker", self.index, wire_msg)
        self.receiver.on_worker_msg(wire_msg, self._on_pull, self._on_push)


class LogicFactory:
    """Wrap ``fn(subtask_index) -> logic`` to build each subtask's logic
    instead of deep-copying one prototype."""

    def __init__(self, fn):
        self.fn = fn

    def __call__(self, i):
        return self.fn(i)


def _instantiate(obj, i):
    """Per-subtask copy of a user object (Flink serializes one per subtask)."""
    if isinstance(obj, LogicFactory):
        return obj(i)
    return copy.deepcopy(obj)


def split_input(data, n: int, partitioner: Optional[Callable] = None) -> List[deque]:
    """Distribute an input over ``n`` worker subtasks.

    ``data`` may be a list of ``n`` per-partition iterables (a source with
    parallelism ``n``), or one iterable dealt round-robin (Flink ``rebalance``)
    or by ``partitioner(record) -> int`` (Flink ``partitionCustom``; the key is
    taken ``% n`` like ``M/FlinkParameterServer.scala:270-274``).
    """
    if isinstance(data, PartitionedInput):
        if len(data.parts) != n:
            raise ValueError(f"input has {len(data.parts)} partitions, expected {n}")
        return list(data.parts)
    parts = [[] for _ in range(n)]
    if partitioner is None:
        for i, rec in enumerate(data):
            parts[i % n].append(rec)
    else:
        for rec in data:
            parts[int(partitioner(rec)) % n].append(rec)
    return parts


class PartitionedInput:
    """Marks an input already split per worker subtask.  Partitions may be
    lazy iterables (generators, ``utils.sleep_blocker.block``); the engine
    consumes them incrementally, interleaved with pull answers."""

    def __init__(self, parts: Sequence[Iterable]):
        self.parts = list(parts)


class LocalRuntime:
    """Single-process runtime for a ``transform`` job (see module docstring)."""

    #: max messages a subtask handles per scheduling turn
    batch = 64

    def __init__(self, iteration_wait_time: Optional[float] = None, output_sink: Optional[Callable] = None):
        self.iteration_wait_time = iteration_wait_time
        self.output_sink = output_sink

    # ------------------------------------------------------------------ setup
    def setup(self, data_parts, worker_logic, ps_logic, param_partitioner, w_in_partition, W, P,
              worker_receiver, worker_sender, ps_receiver, ps_sender, local_workers=None, local_ps=None):
        self.W, self.P = W, P
        self.param_partitioner = param_partitioner
        self.w_in_partition = w_in_partition
        self.outputs: List[Any] = []
        self.workers = {}
        self.servers = {}
        local_workers = range(W) if local_workers is None else local_workers
        local_ps = range(P) if local_ps is None else local_ps
        for w in local_workers:
            t = WorkerTask(w, _instantiate(worker_logic, w), copy.deepcopy(worker_sender),
                           copy.deepcopy(worker_receiver), self)
            t.data = iter(data_parts[w]) if data_parts is not None else None
            self.workers[w] = t
        for p in local_ps:
            self.servers[p] = PSTask(p, _instantiate(ps_logic, p), copy.deepcopy(ps_sender),
                                     copy.deepcopy(ps_receiver), self)
        self._last_activity = time.monotonic()

    def open(self, world_rank=0, world_size=1, device="cpu"):
        for w, t in self.workers.items():
            t.logic.open(RuntimeContext(w, self.W, world_rank, world_size, device, "worker"))
        for p, t in self.servers.items():
            t.logic.open({}, RuntimeContext(p, self.P, world_rank, world_size, device, "ps"))

    # ----------------------------------------------------------------- routing
    def emit_output(self, e):
        if self.output_sink is not None:
            self.output_sink(e)
        else:
            self.outputs.append(e)

    def ps_index(self, msg) -> int:
        return int(self.param_partitioner(msg)) % self.P

    def worker_index(self, msg) -> int:
        k = int(self.w_in_partition(msg))
        if not (0 <= k < self.W):
            raise RuntimeError("Pull answer key should be the partition ID itself!")
        return k

    def route_to_ps(self, msg):
        self.servers[self.ps_index(msg)].inbox.append(msg)

    def route_to_worker(self, msg):
        self.workers[self.worker_index(msg)].answers.append(msg)

    # --------------------------------------------------------------- running
    def _step_local(self) -> bool:
        """One scheduling pass over local subtasks; True if anything ran."""
        progressed = False
        b = self.batch
        for t in self.workers.values():
            ans = t.answers
            n = 0
            while ans and n < b:
                t.handle_answer(ans.popleft())
                n += 1
            m = 0
            src = t.data
            if src is not None:  # lazily consumed input partition
                for rec in src:
                    t.handle_data(rec)
                    m += 1
                    if m >= b:
                        break
                else:
                    t.data = None
            if n or m:
                progressed = True
        for t in self.servers.values():
            inbox = t.inbox
            n = 0
            while inbox and n < b:
                t.handle_msg(inbox.popleft())
                n += 1
            if n:
                progressed = True
        if progressed:
            self._last_activity = time.monotonic()
        return progressed

    def _locally_idle(self) -> bool:
        for t in self.workers.values():
            if t.answers or t.data is not None:
                return False
        for t in self.servers.values():
            if t.inbox:
                return False
        return True

    def _pending_buffers(self) -> int:
        n = 0
        for t in self.workers.values():
            n += t.sender.pending()
        for t in self.servers.values():
            n += t.sender.pending()
        return n

    def _flush_buffers(self):
        for t in self.workers.values():
            if hasattr(t.sender, "flush") and t.sender.pending():
                t.sender.flush(t.emit_to_ps)
        for t in self.servers.values():
            if hasattr(t.sender, "flush") and t.sender.pending():
                t.sender.flush(t.emit_to_worker)

    def _wait_budget(self) -> float:
        return (self.iteration_wait_time or 0) / 1000.0

    def run(self):
        """Run to quiescence, close every subtask, return the output stream."""
        budget = self._wait_budget()
        grace = budget if self.iteration_wait_time is not None else 10.0
        while True:
            if self._step_local():
                continue
            idle = time.monotonic() - self._last_activity
            if self._pending_buffers():
                # buffered combination messages: let their timers flush them
                # (bounded), then flush what is left rather than dropping it
                if self._has_timers() and idle < grace:
                    time.sleep(0.001)
                    continue
                self._flush_buffers()
                continue
            if idle < budget:  # keep alive for user threads
                time.sleep(0.001)
                continue
            break
        self.close()
        return self.outputs

    def _has_timers(self) -> bool:
        from .adapters import CombinationLogic, TimerLogic

        for t in list(self.workers.values()) + list(self.servers.values()):
            s = t.sender
            if isinstance(s, CombinationLogic) and any(isinstance(c, TimerLogic) for c in s.combinables):
                return True
        return False

    def close(self):
        for t in self.workers.values():
            t.logic.close()
        for t in self.servers.values():
            t.logic.close(t.handle)
        for t in list(self.workers.values()) + list(self.servers.values()):
            t.sender.close()
        close = getattr(self.output_sink, "close", None)
        if callable(close):  # a Flink sink's close(): may end the job (utils.testing.SuccessException)
            close()


# ---------------------------------------------------------------------------
# public entry points
def _default_partitioners(P: int):
    def w2ps(msg: WorkerToPS):
        return hash_partition(msg.msg.value.param_id, P)

    def ps2w(msg: PSToWorker):
        return msg.worker_partition_index

    return w2ps, ps2w


def transform(training_data, worker_logic: WorkerLogic, ps_logic: Optional[ParameterServerLogic] = None, *,
              param_init: Optional[Callable] = None, param_update: Optional[Callable] = None,
              param_partitioner: Optional[Callable] = None, w_in_partition: Optional[Callable] = None,
              worker_parallelism: Optional[int] = None, ps_parallelism: Optional[int] = None,
              worker_receiver=None, worker_sender=None, ps_receiver=None, ps_sender=None,
              iteration_wait_time: Optional[float] = None, data_partitioner: Optional[Callable] = None,
              runtime=None, output_sink: Optional[Callable] = None, backend: str = "record",
              comm=None, staleness: int = 0, num_ids: Optional[int] = None, combine: str = "sum",
              graph: bool = False, capacity: Optional[int] = None) -> List[Any]:
    """Run a parameter-server job; returns the ``Left(wout)``/``Right(psout)`` stream.

    Covers the three reference overloads (``M/FlinkParameterServer.scala:62-336``):

    (a) ``param_init`` + ``param_update`` -> ``SimplePSLogic`` (``:62-77``);
    (b) ``ps_logic`` with hash partitioning ``|id| % P`` and Simple adapters
        (``:108-149``);
    (c) fully custom partitioners / wire adapters (``:195-336``).

    ``backend="tensor"`` runs the job on the tensor engine instead
    (``core.tensor_engine``, one process per GPU under torchrun):
    ``training_data`` is this rank's iterable of micro-batches,
    ``worker_logic`` a ``BatchedWorkerLogic``; worker / PS parallelism = at most
    the world size of ``comm`` (default: equal to it); ``staleness`` bounds the micro-batches in flight
    (the ``pullLimit`` analogue, ``tensor_engine.staleness_for_pull_limit``).
    The three overloads map to:

    (a) ``param_init(ids) -> rows`` / ``param_update(old, delta[, ids]) -> new``
        (vectorised torch callables) -> ``DeviceFunctionPSLogic``; ``num_ids``
        sizes a dense shard, ``None`` = a sparse hash-table shard over the whole
        int32 id space; ``combine`` = how repeated pushes of a key in one
        micro-batch meet (``sum`` / ``max`` / ``min`` / ``last`` / ``sequential``);
    (b) ``ps_logic`` = a device PS logic (``ps.device_logics``);
    (c) ``param_partitioner`` = a vectorised ``ids -> shard`` callable or an
        ``owner[num_ids]`` tensor (the shard lookup the device path routes by).

    Arguments the tensor engine cannot honour raise ``ValueError`` instead of
    being dropped: wire adapters (the wire is SoA tensors; batching =
    ``core.microbatch.MicroBatcher``), ``w_in_partition`` (answers always return
    to the requester), ``data_partitioner`` / ``runtime`` (each rank passes its
    own source), parallelisms above the world size (``worker_parallelism`` /
    ``ps_parallelism`` below it leave ranks without a worker / shard).  ``graph`` / ``capacity``
    (tensor backend): hipGraph-replayed steps / fixed-shape plans (``TensorRuntime``).
    """
    if backend == "tensor":
        return _transform_tensor(training_data, worker_logic, ps_logic, param_init, param_update, param_partitioner,
                                 w_in_partition, worker_parallelism, ps_parallelism,
                                 dict(worker_receiver=worker_receiver, worker_sender=worker_sender,
                                      ps_receiver=ps_receiver, ps_sender=ps_sender,
                                      data_partitioner=data_partitioner, runtime=runtime),
                                 iteration_wait_time, output_sink, comm, staleness, num_ids, combine, graph, capacity)
    if graph or capacity is not None:
        raise ValueError("graph / capacity configure the tensor backend (backend='tensor')")
    if backend != "record":
        raise ValueError(f"backend must be 'record' or 'tensor', not {backend!r}")
    if num_ids is not None or combine != "sum" or comm is not None or staleness:
        raise ValueError("num_ids / combine / comm / staleness are tensor-backend arguments")
    if ps_logic is None:
        if param_init is None or param_update is None:
            raise ValueError("give ps_logic or (param_init, param_update)")
        ps_logic = SimplePSLogic(param_init, param_update)
    W, P = int(worker_parallelism or 1), int(ps_parallelism or 1)
    dp, dw = _default_partitioners(P)
    param_partitioner = param_partitioner or dp
    w_in_partition = w_in_partition or dw
    worker_receiver = worker_receiver or SimpleWorkerReceiver()
    worker_sender = worker_sender or SimpleWorkerSender()
    ps_receiver = ps_receiver or SimplePSReceiver()
    ps_sender = ps_sender or SimplePSSender()
    if runtime is None:
        runtime = LocalRuntime(iteration_wait_time, output_sink)
    else:
        runtime.iteration_wait_time = iteration_wait_time if iteration_wait_time is not None else \
            runtime.iteration_wait_time
        if output_sink is not None:
            runtime.output_sink = output_sink
    return runtime.execute(training_data, worker_logic, ps_logic, param_partitioner, w_in_partition, W, P,
                           worker_receiver, worker_sender, ps_receiver, ps_sender, data_partitioner) \
        if hasattr(runtime, "execute") else _execute_local(runtime, training_data, worker_logic, ps_logic,
                                                            param_partitioner, w_in_partition, W, P,
                                                            worker_receiver, worker_sender, ps_receiver,
                                                            ps_sender, data_partitioner)


def _transform_tensor(training_data, worker_logic, ps_logic, param_init, param_update, param_partitioner,
                      w_in_partition, worker_parallelism, ps_parallelism, adapters, iteration_wait_time, output_sink,
                      comm, staleness, num_ids, combine, graph=False, capacity=None):
    """``transform(backend="tensor")``: map the overloads onto the tensor engine
    (see ``transform``), refusing what it cannot honour."""
    import torch

    from ..api.batched import BatchedWorkerLogic
    from ..parallel.comm import Comm
    from ..ps.device_logics import DeviceFunctionPSLogic, DevicePSLogic
    from .tensor_engine import transform_tensor

    given = sorted(k for k, v in adapters.items() if v is not None)
    if given:
        raise ValueError(f"backend='tensor' does not take {given}: its wire format is fixed (SoA tensors over "
                         "all-to-alls), micro-batching is core.microbatch.MicroBatcher, and each rank passes its own "
                         "source iterable")
    if w_in_partition is not None:
        raise ValueError("backend='tensor' always answers a pull to the worker that sent it; w_in_partition "
                         "cannot be honoured")
    if not isinstance(worker_logic, BatchedWorkerLogic):
        raise TypeError("backend='tensor' needs a BatchedWorkerLogic (api.batched)")
    comm = comm or Comm()
    for name, par in (("worker_parallelism", worker_parallelism), ("ps_parallelism", ps_parallelism)):
        if par is not None and not 1 <= int(par) <= comm.world:
            raise ValueError(f"backend='tensor': {name}={par} but the job has {comm.world} ranks (at most one "
                             "worker and one PS shard per rank)")
    if ps_logic is None:
        if param_init is None or param_update is None:
            raise ValueError("give ps_logic or (param_init, param_update)")
        probe = torch.as_tensor(param_init(torch.zeros(1, dtype=torch.int64)))
        dim = int(probe.reshape(1, -1).shape[1])
        if param_partitioner is not None and num_ids is None:
            raise ValueError("a custom param_partitioner on the tensor backend needs num_ids (a dense id space)")
        # the parameter type P follows the init: fp64 rows (and wire) for a double init
        f64 = probe.dtype == torch.float64
        ps_logic = DeviceFunctionPSLogic(dim, param_init, param_update, num_ids, combine=combine,
                                         partition=param_partitioner if param_partitioner is not None else "hash",
                                         dtype=torch.float64 if f64 else torch.float32,
                                         wire_dtype="fp64" if f64 else "fp32")
    else:
        if param_init is not None or param_update is not None:
            raise ValueError("give ps_logic or (param_init, param_update), not both")
        if num_ids is not None or combine != "sum":
            raise ValueError("num_ids / combine configure overload (a); set them on the device logic instead")
        if not isinstance(ps_logic, DevicePSLogic):
            raise TypeError("backend='tensor' needs a device PS logic (ps.device_logics)")
        if param_partitioner is not None:
            if ps_logic.sparse or ps_logic._given[0] is not None:
                raise ValueError("param_partitioner needs a dense shard allocated by the logic")
            ps_logic.partition = param_partitioner
    return transform_tensor(training_data, worker_logic, ps_logic, comm=comm, staleness=staleness,
                            iteration_wait_time=iteration_wait_time, output_sink=output_sink, graph=graph,
                            capacity=capacity, worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism)


def _execute_local(rt: LocalRuntime, training_data, worker_logic, ps_logic, param_partitioner, w_in_partition,
                   W, P, worker_receiver, worker_sender, ps_receiver, ps_sender, data_partitioner):
    parts = split_input(training_data, W, data_partitioner)
    rt.setup(parts, worker_logic, ps_logic, param_partitioner, w_in_partition, W, P,
             worker_receiver, worker_sender, ps_receiver, ps_sender)
    rt.open()
    return rt.run()


# ---------------------------------------------------------------- model load
class _EOF:
    """Model-load end marker (``case class EOF()`` in the reference)."""

    __slots__ = ()

    def __eq__(self, other):
        return isinstance(other, _EOF)

    def __hash__(self):
        return 0x0E0F

    def __repr__(self):
        return "EOF()"


EOF_MARK = _EOF()


class _Param:
    """``Parameter(id, p)`` wrapper of the double-load protocol."""

    __slots__ = ("param_id", "value")

    def __init__(self, param_id, value):
        self.param_id = param_id
        self.value = value

    def __getstate__(self):
        return (self.param_id, self.value)

    def __setstate__(self, s):
        self.param_id, self.value = s


class _UnwrapClient(ParameterServerClient):
    """User-facing client that wraps pushed deltas (``wrapPSClient``)."""

    __slots__ = ("ps", "wrap")

    def __init__(self, wrap):
        self.ps = None
        self.wrap = wrap

    def pull(self, param_id):
        self.ps.pull(param_id)

    def push(self, param_id, delta):
        self.ps.push(param_id, self.wrap(param_id, delta))

    def output(self, out):
        self.ps.output(out)


class _UnwrapPS(ParameterServer):
    __slots__ = ("ps", "wrap")

    def __init__(self, wrap):
        self.ps = None
        self.wrap = wrap

    def answer_pull(self, param_id, value, worker_partition_index):
        self.ps.answer_pull(param_id, self.wrap(param_id, value), worker_partition_index)

    def output(self, out):
        self.ps.output(out)


class ModelLoadWorkerLogic(WorkerLogic):
    """Worker side of ``transformWithModelLoad`` (``M/FlinkParameterServer.scala:435-482``).

    Inputs are ``Left(Right((id, p)))`` model records, ``Left(Left(EOF))`` and
    ``Right(x)`` training data.  Model records are pushed to their PS; data is
    buffered until this worker saw EOF; EOF is broadcast to every PS index.
    ``double=True`` implements ``transformWithDoubleModelLoad`` (``:607-816``):
    ``("ps", (id, p))`` goes to the PS, ``("worker", (id, p))`` to the
    worker's ``update_model``.
    """

    def __init__(self, worker_logic, ps_parallelism, double=False):
        self.worker_logic = worker_logic
        self.ps_parallelism = ps_parallelism
        self.double = double
        self.received_eof = False
        self.buffer = []
        wrap = (lambda pid, d: _Param(pid, d)) if double else (lambda pid, d: Right(d))
        self._client = _UnwrapClient(wrap)

    def open(self, ctx):
        self.worker_logic.open(ctx)

    def on_recv(self, rec, ps):
        c = self._client
        c.ps = ps
        kind, payload = rec
        if kind == "data":
            if self.received_eof:
                self.worker_logic.on_recv(payload, c)
            else:
                self.buffer.append(payload)
        elif kind == "eof":
            self.received_eof = True
            eof = EOF_MARK if self.double else Left(EOF_MARK)
            for p in range(self.ps_parallelism):
                ps.push(p, eof)
            buf, self.buffer = self.buffer, []
            for x in buf:
                self.worker_logic.on_recv(x, c)
        elif kind == "ps":
            pid, val = payload
            ps.push(pid, _Param(pid, val) if self.double else Right(val))
        elif kind == "worker":
            pid, val = payload
            self.worker_logic.update_model(pid, val)
        else:
            raise ValueError(kind)

    def on_pull_recv(self, param_id, value, ps):
        self._client.ps = ps
        if self.double:
            if isinstance(value, _Param):
                self.worker_logic.on_pull_recv(param_id, value.value, self._client)
            # keep-alive EOF answers are ignored (:710-711)
        else:
            if isinstance(value, Right):
                self.worker_logic.on_pull_recv(param_id, value.value, self._client)
            else:
                raise RuntimeError("PS should not send EOF pull answers")

    def close(self):
        self.worker_logic.close()


class ModelLoadPSLogic(ParameterServerLogic):
    """PS side of the model-load protocol (``M/FlinkParameterServer.scala:506-545``):
    pulls are buffered until ``worker_parallelism`` EOFs arrived, then replayed."""

    def __init__(self, ps_logic, worker_parallelism, double=False):
        self.ps_logic = ps_logic
        self.worker_parallelism = worker_parallelism
        self.eof_count_down = worker_parallelism
        self.pull_buffer = []
        self.double = double
        wrap = (lambda pid, v: _Param(pid, v)) if double else (lambda pid, v: Right(v))
        self._ps = _UnwrapPS(wrap)

    def open(self, config, ctx):
        self.ps_logic.open(config, ctx)

    def on_pull_recv(self, param_id, worker_partition_index, ps):
        if self.eof_count_down == 0:
            self._ps.ps = ps
            self.ps_logic.on_pull_recv(param_id, worker_partition_index, self._ps)
        else:
            self.pull_buffer.append((param_id, worker_partition_index))

    def on_push_recv(self, param_id, delta, ps):
        self._ps.ps = ps
        is_eof = (delta == EOF_MARK) if self.double else (isinstance(delta, Left))
        if is_eof:
            self.eof_count_down -= 1
            if self.eof_count_down == 0:
                buf, self.pull_buffer = self.pull_buffer, []
                for pid, widx in buf:
                    self.ps_logic.on_pull_recv(pid, widx, self._ps)
        else:
            value = delta.value
            if self.double and self.eof_count_down > 0:
                # keep-alive so the idle timeout does not fire during load (:780-783)
                ps.answer_pull(param_id, EOF_MARK, param_id % self.worker_parallelism)
            self.ps_logic.on_push_recv(param_id, value, self._ps)

    def close(self, ps):
        self._ps.ps = ps
        self.ps_logic.close(self._ps)


def _model_load_inputs(model, training_data, W, data_partitioner, double):
    model = list(model)
    if len(model) < W:
        raise RuntimeError("There must be a parameter per model partition when loading model.")
    mparts = [[] for _ in range(W)]
    for i, rec in enumerate(model):
        if double:
            kind = "ps" if rec.is_left else "worker"
            mparts[i % W].append((kind, tuple(rec.value)))
        else:
            mparts[i % W].append(("ps", tuple(rec)))
    dparts = split_input(training_data, W, data_partitioner)
    parts = []
    for w in range(W):
        ms, ds = mparts[w], list(dparts[w])
        merged = []
        # interleave model and data (both inputs race in Flink); this worker's
        # EOF follows its last model record
        for i in range(max(len(ms), len(ds))):
            if i < len(ms):
                merged.append(ms[i])
                if i == len(ms) - 1:
                    merged.append(("eof", None))
            if i < len(ds):
                merged.append(("data", ds[i]))
        parts.append(merged)
    return PartitionedInput(parts)


def _wrap_partitioners(param_partitioner, w_in_partition, double):
    from .messages import Pull, Push, PullAnswer

    def w2ps(msg: WorkerToPS):
        m = msg.msg
        inner = m.value
        if m.is_right:
            d = inner.delta
            if double:
                if d == EOF_MARK:
                    return inner.param_id
                return param_partitioner(WorkerToPS(msg.worker_partition_index, Right(Push(inner.param_id, d.value))))
            if isinstance(d, Left):
                return inner.param_id
            return param_partitioner(WorkerToPS(msg.worker_partition_index, Right(Push(inner.param_id, d.value))))
        return param_partitioner(msg)

    def ps2w(msg: PSToWorker):
        v = msg.msg.param
        if double:
            if v == EOF_MARK:
                return msg.worker_partition_index
            return w_in_partition(PSToWorker(msg.worker_partition_index, PullAnswer(msg.msg.param_id, v.value)))
        return w_in_partition(PSToWorker(msg.worker_partition_index, PullAnswer(msg.msg.param_id, v.value)))

    return w2ps, ps2w


def transform_with_model_load(model: Iterable, training_data, worker_logic, ps_logic, *,
                              param_partitioner=None, w_in_partition=None, worker_parallelism=1,
                              ps_parallelism=1, iteration_wait_time=None, data_partitioner=None,
                              runtime=None, output_sink=None):
    """Warm start from a model stream of ``(id, p)`` (``M/FlinkParameterServer.scala:377-566``).

    Model records are pushed into the (empty) PS store before any pull is
    served.  ``ps_logic`` must accept a push for a key it has not seen.
    """
    W, P = int(worker_parallelism or 1), int(ps_parallelism or 1)
    dp, dw = _default_partitioners(P)
    w2ps, ps2w = _wrap_partitioners(param_partitioner or dp, w_in_partition or dw, double=False)
    inputs = _model_load_inputs(model, training_data, W, data_partitioner, double=False)
    return transform(inputs, ModelLoadWorkerLogic(worker_logic, P), ModelLoadPSLogic(ps_logic, W),
                     param_partitioner=w2ps, w_in_partition=ps2w, worker_parallelism=W, ps_parallelism=P,
                     iteration_wait_time=iteration_wait_time, runtime=runtime, output_sink=output_sink)


def transform_with_double_model_load(model: Iterable, training_data, worker_logic, ps_logic, *,
                                     param_partitioner=None, w_in_partition=None, worker_parallelism=1,
                                     ps_parallelism=1, iteration_wait_time=None, data_partitioner=None,
                                     runtime=None, output_sink=None):
    """Warm start of PS model (``Left((id, p))``) and worker-resident model
    (``Right((id, p))``, delivered to ``worker_logic.update_model`` of the worker
    receiving the record) (``M/FlinkParameterServer.scala:607-816``)."""
    W, P = int(worker_parallelism or 1), int(ps_parallelism or 1)
    dp, dw = _default_partitioners(P)
    w2ps, ps2w = _wrap_partitioners(param_partitioner or dp, w_in_partition or dw, double=True)
    inputs = _model_load_inputs(model, training_data, W, data_partitioner, double=True)
    return transform(inputs, ModelLoadWorkerLogic(worker_logic, P, double=True),
                     ModelLoadPSLogic(ps_logic, W, double=True),
                     param_partitioner=w2ps, w_in_partition=ps2w, worker_parallelism=W, ps_parallelism=P,
                     iteration_wait_time=iteration_wait_time, runtime=runtime, output_sink=output_sink)


class FlinkParameterServer:
    """Scala-named facade: ``FlinkParameterServer.transform(...)`` etc."""

    transform = staticmethod(transform)
    transformWithModelLoad = staticmethod(transform_with_model_load)
    transformWithDoubleModelLoad = staticmethod(transform_with_double_model_load)
