"""Tensor engine: ``transform`` on device micro-batches over RCCL.

The reference runs user ``WorkerLogic`` / ``ParameterServerLogic`` callbacks
inside a Flink streaming iteration (``M/FlinkParameterServer.scala:195-336``).
Here the same roles run on every GPU rank (one process per GPU, ``torchrun``),
with worker ``r`` and PS shard ``r`` co-located on rank ``r``:

* the user's ``BatchedWorkerLogic`` (``api/batched.py``) turns each micro-batch
  into pull requests and each answer into pushes / outputs;
* a device PS logic (``ps/device_logics.py``) owns an HBM shard; pulls and
  pushes travel as all-to-alls (``parallel.tensor_ps.TensorPS``);
* ``parallel.staleness.BoundedStalenessPipeline`` overlaps micro-batches with
  at most ``staleness`` un-applied pushes behind any served pull -- the
  ``pullLimit`` bound (``M/WorkerLogic.scala:176-225``); counts of micro-batch
  ``k+1`` are exchanged while ``k`` computes, so the host never stalls the
  device on split sizes;
* outputs: ``Left(worker output)`` / ``Right(PS output)`` in micro-batch order
  (``M/FlinkParameterServer.scala:319-328``), handed to ``output_sink`` as they
  happen (device tensors; ``FoldSink`` folds them last-writer-wins on device);
* end of input: each rank's source may hold a different number of
  micro-batches; an exhausted rank keeps taking part with empty micro-batches
  until every rank is exhausted (the flag rides on the count exchange), then
  ``on_eof`` may replay more (offline epochs), then ``close``;
* model load (``transformWithModelLoad`` / ``...DoubleModelLoad``,
  ``M/FlinkParameterServer.scala:377-816``): ``(id, value)`` records of every
  rank are routed to their owning shards (one ``set``-push) before the first
  pull; ``Right`` records go to the local worker's ``update_model_batch``.
  Stream order + the collective replace the reference's EOF counting.

``transform(..., backend="tensor")`` in ``core.engine`` dispatches here.
"""
from __future__ import annotations

import threading
import queue
from typing import Any, Callable, Iterable, Iterator, List, Optional, Sequence

import torch

from ..api.batched import BatchedPSClient, BatchedWorkerLogic, PulledBatch
from ..api.logic import RuntimeContext
from ..parallel.comm import Comm
from ..parallel.staleness import BoundedStalenessPipeline
from ..ps.device_logics import DevicePSLogic
from ..utils.metrics import Counters
from ..utils.tracing import stage
from .messages import Left, Right
from .step_graph import StepGraphs


def staleness_for_pull_limit(pull_limit: int, micro_batch: int) -> int:
    """Micro-batches that may be in flight for a per-worker ``pullLimit`` when
    each micro-batch issues ``micro_batch`` pulls (at least one: synchronous)."""
    return max(0, -(-int(pull_limit) // max(int(micro_batch), 1)) - 1)


class _Request:
    __slots__ = ("keys", "payload", "off", "n", "presence")

    def __init__(self, keys, payload, off, n, presence=None):
        self.keys, self.payload, self.off, self.n = keys, payload, off, n
        self.presence = presence


class _Client(BatchedPSClient):
    """The ``BatchedPSClient`` handed to the worker (one per rank)."""

    def __init__(self, rt: "TensorRuntime"):
        self.rt = rt
        self._requests: Optional[List[_Request]] = None
        self._n = 0
        # answer context
        self._plan = None
        self._req: Optional[_Request] = None
        self._acc: Optional[torch.Tensor] = None
        self._mask: Optional[torch.Tensor] = None
        self._direct: Optional[torch.Tensor] = None
        self._applied = False  # the worker added this answer's push to the table itself
        self._seq: List[tuple] = []  # (pos, deltas, mask) per push, combine="sequential"
        self._arb_keys: List[torch.Tensor] = []
        self._arb_vals: List[torch.Tensor] = []

    # --------------------------------------------------------------- pulls
    def pull(self, keys, payload=None, presence=None):
        """``presence`` (optional, a hint): ``(flags uint8[key space], ready event)`` -- which
        keys of the table occur in ``keys``, computed by the worker anyway (e.g. by its
        partition pass); a plan over the whole key space (identity plan) then skips its
        own marking pass.  Used only when this is the micro-batch's only request."""
        if self._requests is None:
            raise RuntimeError("pull() is only valid inside on_recv_batch")
        keys = torch.as_tensor(keys).reshape(-1)
        self._requests.append(_Request(keys, payload, self._n, keys.numel(), presence))
        self._n += keys.numel()

    # --------------------------------------------------------------- pushes
    def _dim(self):
        return self.rt.ps_logic.dim

    def _ensure_acc(self):
        if self._acc is None:
            U = self._plan.n_unique
            dev = self.rt.device
            dtype = self.rt.ps_logic.dtype
            if self._direct is not None:  # a previous push_unique handed its buffer through
                self._acc = self._direct.to(dtype).clone()
                self._direct = None
                self._mask = torch.ones(U, dtype=torch.bool, device=dev)
            else:
                self._acc = torch.zeros((U, self._dim()), dtype=dtype, device=dev)
                self._mask = torch.zeros(U, dtype=torch.bool, device=dev)

    def push(self, deltas, mask=None):
        """One delta row per request of the pull being answered."""
        if self._req is None:
            raise RuntimeError("push() is only valid inside on_pull_recv_batch")
        r = self._req
        d = deltas.reshape(r.n, self._dim()).to(device=self.rt.device)
        pos = self._plan.pos[r.off:r.off + r.n].long()
        if mask is not None:
            mask = mask.to(device=self.rt.device, dtype=torch.bool).reshape(-1)
        self._accumulate(pos, d, mask)

    def _accumulate(self, pos, d, mask):
        """Fold request deltas into the per-unique-key push buffer with the
        logic's ``combine`` rule (``sum`` unless the PS rule says otherwise)."""
        comb = self.rt.ps_logic.combine
        if comb == "sequential":  # kept per request; TensorRuntime._push sends one round per repeat
            self._seq.append((pos, d, mask))
            return
        self._ensure_acc()
        if comb in ("max", "min"):
            U = self._plan.n_unique
            idx = pos if mask is None else torch.where(mask, pos, torch.full_like(pos, U))
            tmp = torch.zeros((U + 1, self._dim()), dtype=self._acc.dtype, device=self._acc.device)
            tmp.scatter_reduce_(0, idx.view(-1, 1).expand(-1, self._dim()), d.to(tmp.dtype),
                                reduce="amax" if comb == "max" else "amin", include_self=False)
            hit = torch.zeros(U + 1, dtype=torch.bool, device=pos.device).index_fill_(0, idx, True)
            tmp, hit = tmp[:U], hit[:U]
            both = torch.maximum(self._acc, tmp) if comb == "max" else torch.minimum(self._acc, tmp)
            self._acc = torch.where((hit & self._mask).view(-1, 1), both,
                                    torch.where(hit.view(-1, 1), tmp, self._acc))
            self._mask |= hit
        elif self.rt.ps_logic.op == "set" or comb == "last":  # last writer wins, in request order
            if pos.numel() == 0:  # an empty request: nothing to write (d may be [0, D] with U > 0)
                return
            rid = torch.arange(pos.numel(), device=pos.device)
            if mask is not None:
                rid = torch.where(mask, rid, torch.full_like(rid, -1))
            last = torch.full((self._plan.n_unique,), -1, dtype=torch.int64, device=pos.device)
            last.scatter_reduce_(0, pos, rid, reduce="amax")
            hit = last >= 0  # (no boolean indexing: the step stays free of host syncs)
            self._acc = torch.where(hit.view(-1, 1), d[last.clamp_min(0)].to(self._acc.dtype), self._acc)
            self._mask |= hit
        else:
            if mask is not None:
                d = d * mask.view(-1, 1).to(d.dtype)
                hits = torch.zeros(self._mask.numel(), dtype=torch.int32, device=pos.device)
                hits.index_add_(0, pos, mask.to(torch.int32))
                self._mask |= hits > 0
            else:
                self._mask.index_fill_(0, pos, True)
            self._acc.index_add_(0, pos, d.to(self._acc.dtype))

    def push_unique(self, deltas, mask=None):
        """Pre-reduced ``[U, D]`` deltas for the unique keys of the answered pull."""
        if self._plan is None:
            raise RuntimeError("push_unique() is only valid inside on_pull_recv_batch")
        U = self._plan.n_unique
        d = deltas.reshape(U, self._dim())
        if self.rt.ps_logic.combine != "sum":
            if mask is not None:
                mask = mask.to(device=d.device, dtype=torch.bool).reshape(-1)
            self._accumulate(torch.arange(U, device=d.device), d, mask)
            return
        if self._acc is None and self._direct is None and mask is None:
            self._direct = d  # fast path: the worker's buffer goes on the wire as is
            return
        self._ensure_acc()
        if mask is None:
            mask = torch.ones(U, dtype=torch.bool, device=d.device)
        mask = mask.to(dtype=torch.bool).reshape(-1)
        if self.rt.ps_logic.op == "set":
            self._acc = torch.where(mask.view(-1, 1), d.to(self._acc.dtype), self._acc)
        else:
            self._acc += d.to(self._acc.dtype) * mask.view(-1, 1).to(self._acc.dtype)
        self._mask |= mask

    def local_push_target(self, in_place: bool = False):
        plan = self._plan
        if plan is None:
            raise RuntimeError("local_push_target() is only valid inside on_pull_recv_batch")
        rt, logic = self.rt, self.rt.ps_logic
        ps = logic.ps if logic is not None else None
        if ps is None or rt.comm.world != 1 or getattr(rt.comm, "loopback", False) or logic.locking:
            return None
        t = ps.table
        if (logic.op != "add" or logic.combine != "sum" or logic.emit == "push" or ps.masked_push
                or getattr(t, "optimizer", "") != "add" or getattr(t, "sparse", False) or plan.fixed
                or t.weight.dtype != torch.float32 or plan.recv_rows is None
                or (self._served_is_table(plan) and not in_place)):
            return None
        return t.weight, plan.recv_rows

    def _served_is_table(self, plan) -> bool:
        """A zero-copy serve hands the table itself out: a push into it would be read
        back by the same micro-batch."""
        return bool(getattr(plan, "zero_copy", False))

    def push_applied(self) -> None:
        if self._plan is None:
            raise RuntimeError("push_applied() is only valid inside on_pull_recv_batch")
        self._applied = True

    def push_keys(self, keys, deltas):
        if not self.rt.worker_logic.arbitrary_pushes:
            raise RuntimeError("push_keys needs the worker class to declare arbitrary_pushes = True")
        self._arb_keys.append(torch.as_tensor(keys, device=self.rt.device).reshape(-1))
        self._arb_vals.append(deltas.reshape(-1, self._dim()).to(device=self.rt.device, dtype=torch.float32))

    # --------------------------------------------------------------- outputs
    def output(self, out):
        self.rt._emit(Left(out))


class TensorRuntime:
    """Per-rank driver of a tensor-engine job (see module docstring)."""

    def __init__(self, comm: Optional[Comm] = None, staleness: int = 0, iteration_wait_time: Optional[float] = None,
                 output_sink: Optional[Callable[[Any], None]] = None, lookahead: Optional[bool] = None,
                 graph: bool = False, capacity: Optional[int] = None, worker_parallelism: Optional[int] = None,
                 ps_parallelism: Optional[int] = None, owner_stream: Optional[bool] = None):
        """``graph``: replay fixed-shape micro-batch steps from captured hipGraphs
        (``core.step_graph``: static plans at world 1, fixed-shape plans over RCCL at
        world > 1, a ``graph_safe`` worker).  ``capacity``: the most keys this rank
        pulls per micro-batch -- fixed-shape plans (``TensorPS.capacity``: no host
        copy of split sizes; required by ``graph`` at world > 1).

        ``worker_parallelism`` / ``ps_parallelism`` (each <= the world, default the
        world): ranks ``>= worker_parallelism`` run no worker input (they still join
        every collective), ranks ``>= ps_parallelism`` hold no PS shard -- the
        reference's independent ``workerParallelism`` / ``psParallelism``
        (``M/FlinkParameterServer.scala:126-138``: shard ``|id| % psParallelism``)."""
        self.comm = comm or Comm()
        W = self.comm.world
        self.worker_parallelism = int(worker_parallelism or W)
        self.ps_parallelism = int(ps_parallelism or W)
        for name, v in (("worker_parallelism", self.worker_parallelism), ("ps_parallelism", self.ps_parallelism)):
            if not 1 <= v <= W:
                raise ValueError(f"{name}={v} on a job of {W} ranks: need 1 <= {name} <= ranks")
        self.device = self.comm.device
        self.staleness = int(staleness)
        self.lookahead = lookahead
        self.iteration_wait_time = iteration_wait_time
        self.output_sink = output_sink
        self.outputs: List[Any] = []
        self.counters = Counters()
        self.timer = None
        self.worker_logic: Optional[BatchedWorkerLogic] = None
        self.ps_logic: Optional[DevicePSLogic] = None
        self._started = False
        self.graph = bool(graph)
        self.capacity = capacity
        #: the PS pipeline's owner stream (``parallel.staleness``): None = where it applies;
        #: False = the interleaved single-stream schedule (latency-bound workers)
        self.owner_stream = owner_stream
        self.graphs: Optional[StepGraphs] = None
        self._capture_emits: Optional[List[Any]] = None

    # ------------------------------------------------------------------ setup
    def start(self, worker_logic: BatchedWorkerLogic, ps_logic: DevicePSLogic) -> "TensorRuntime":
        """Open both logics on this rank (``open`` of the reference's operators)."""
        self.worker_logic, self.ps_logic = worker_logic, ps_logic
        c = self.comm
        if self.ps_parallelism != c.world:
            if ps_logic.locking or ps_logic.sparse:
                raise ValueError("ps_parallelism < ranks needs a dense, non-locking PS logic")
            ps_logic.ps_parallelism = self.ps_parallelism
        ps_logic.open(c)
        ps_logic.ps.timer = self.timer
        # a rank past worker_parallelism runs no worker subtask: its context index is its
        # own rank (>= worker_parallelism), which no real subtask uses
        worker_logic.open(RuntimeContext(c.rank, self.worker_parallelism, c.rank,
                                         c.world, self.device, "worker", comm=c))
        self.client = _Client(self)
        if ps_logic.locking:
            self.pipe = None
        else:
            # world 1 on the GPU: static plans, so no micro-batch waits on the device;
            # fixed-shape plans wherever a capacity is given and static plans are not used
            ps_logic.ps.capacity = self.capacity
            ps_logic.ps.static = c.world == 1 and self.device.type == "cuda" and \
                (self.capacity is None or not getattr(c, "loopback", False))
            self.pipe = BoundedStalenessPipeline(ps_logic.ps, self._compute, self.staleness,
                                                 lookahead=self.lookahead,
                                                 owner_stream=False if self.graph else self.owner_stream,
                                                 interleave=False if self.graph else None)
        self._started = True
        if self.graph:
            self.graphs = StepGraphs(self)
            why = self.graphs.why_not()
            if why is not None:
                raise ValueError(f"TensorRuntime(graph=True) cannot capture this job's steps: {why}")
            ps_logic.ps.dedup.clear_after = True
        return self

    def set_timer(self, timer) -> None:
        if timer is not None and self.graphs is not None:
            raise ValueError("a stage timer cannot time captured (graph=True) steps")
        self.timer = timer
        if self.ps_logic is not None and self.ps_logic.ps is not None:
            self.ps_logic.ps.timer = timer

    # ------------------------------------------------------------ model load
    @staticmethod
    def _as_tensors(records, dim: Optional[int], device):
        """``(ids, values)`` tensors from a tensor pair or ``(id, value)`` records."""
        if isinstance(records, tuple) and len(records) == 2 and torch.is_tensor(records[0]):
            ids, vals = records
        else:
            recs = list(records)
            ids = torch.tensor([int(r[0]) for r in recs], dtype=torch.int64)
            vals = torch.tensor([[float(v) for v in r[1]] if hasattr(r[1], "__len__") else [float(r[1])]
                                 for r in recs], dtype=torch.float32)
            if not recs:
                vals = torch.zeros((0, dim or 1))
        ids = ids.to(device).reshape(-1)
        vals = vals.to(device=device, dtype=torch.float32).reshape(ids.numel(), -1)
        if dim is not None and vals.shape[1] != dim:
            raise ValueError(f"model rows have {vals.shape[1]} values, the table has {dim}")
        return ids, vals

    def load_model(self, ps_records=None, worker_records=None) -> None:
        """Warm start (collective): ``ps_records`` -- this rank's ``(id, value)``
        records of the PS model (routed to their owners); ``worker_records`` --
        records for this rank's worker-resident model (``update_model_batch``).
        Each is ``(ids, values)`` tensors or an iterable of ``(id, value)``."""
        dim = self.ps_logic.dim
        ps_t = self._as_tensors(ps_records if ps_records is not None else [], dim, self.device)
        with stage("engine.model-load", self.timer):
            self.ps_logic.ps.load(*ps_t)
            if worker_records is not None:
                self.worker_logic.update_model_batch(*self._as_tensors(worker_records, None, self.device))
        self.comm.barrier()  # every shard holds its model before the first pull is served

    # --------------------------------------------------------------- running
    def _emit(self, e) -> None:
        if self._capture_emits is not None:  # capturing a step: re-emitted after every replay
            self._capture_emits.append(e)
            return
        if self.output_sink is not None:
            self.output_sink(e)
        else:
            self.outputs.append(e)

    def submit(self, batch: Any, flag: int = 0) -> None:
        """One micro-batch of this rank (collective: all ranks submit in lockstep;
        ``batch=None`` takes part without data).  A rank ``>= worker_parallelism`` has
        no worker subtask and must submit ``None``."""
        if batch is not None and self.comm.rank >= self.worker_parallelism:
            raise ValueError(f"rank {self.comm.rank} runs no worker (worker_parallelism="
                             f"{self.worker_parallelism}): submit None here and give its input to a worker rank")
        if self.graphs is not None and self.graphs.submit(batch, flag):
            return
        self._submit_eager(batch, flag)

    def _submit_eager(self, batch: Any, flag: int = 0) -> None:
        c = self.client
        c._requests, c._n = [], 0
        if batch is not None:
            with stage("engine.on_recv", self.timer):
                self.worker_logic.on_recv_batch(batch, c)
        reqs, c._requests = c._requests, None
        if reqs:
            # one key tensor as the worker gave it (no int64 round trip when every
            # request is int32: at 4M keys per micro-batch the conversions and the
            # copy cost ~40 us, profiles/r3_pa_ps_path_kernel_stats.csv)
            kd = torch.int32 if all(r.keys.dtype == torch.int32 for r in reqs) else torch.int64
            keys = reqs[0].keys.to(device=self.device, dtype=kd) if len(reqs) == 1 else \
                torch.cat([r.keys.to(device=self.device, dtype=kd) for r in reqs])
        else:
            keys = torch.zeros(0, dtype=torch.int64, device=self.device)
        self.counters.add("micro_batches", 1 if batch is not None else 0)
        self.counters.add("pulls", keys.numel())
        if self.pipe is None:
            self._locked_step(keys, reqs, flag)
        else:
            hint = reqs[0].presence if len(reqs) == 1 else None
            self.pipe.submit(keys, reqs, flag, presence=hint)

    def _compute(self, rows, plan, reqs):
        c = self.client
        c._plan, c._acc, c._mask, c._direct = plan, None, None, None
        c._applied = False
        c._arb_keys, c._arb_vals, c._seq = [], [], []
        with stage("engine.on_pull_recv", self.timer):
            for r in reqs:
                c._req = r
                self.worker_logic.on_pull_recv_batch(
                    PulledBatch(r.keys, rows, plan.pos[r.off:r.off + r.n], r.payload,
                                identity=plan.identity and len(reqs) == 1), c)
        c._req = None
        self._push(plan, c)
        c._plan = None
        return None, None

    def _push(self, plan, c) -> None:
        if not self.worker_logic.pushes:  # a query-only worker: no push round at all
            return
        ps = self.ps_logic.ps
        if c._applied:  # the worker's kernel added the push to the (local) table already
            if c._direct is not None or c._acc is not None or c._seq:
                raise RuntimeError("push_applied() and push() on the same answer")
            ps.note_local_push(plan)
            self.counters.add("pushes", plan.n_unique)
        elif self.ps_logic.combine == "sequential":
            self._push_rounds(plan, c)
        elif c._direct is not None:
            deltas, mask = c._direct, None
        elif c._acc is not None:
            deltas, mask = c._acc, c._mask
        else:  # nothing pushed here; the push all-to-all is collective all the same
            deltas = torch.zeros((plan.n_unique, self.ps_logic.dim), dtype=self.ps_logic.dtype, device=self.device)
            mask = torch.zeros(plan.n_unique, dtype=torch.bool, device=self.device)
        emit = self.ps_logic.emit == "push"
        if self.ps_logic.combine != "sequential" and not c._applied:
            updated = ps.push(plan, deltas, lr=self.ps_logic.lr, return_updated=emit, mask=mask)
            self.counters.add("pushes", plan.n_unique)
            for out in self.ps_logic.after_push(updated):
                self._emit(Right(out))
        if self.worker_logic.arbitrary_pushes:
            keys = torch.cat(c._arb_keys) if c._arb_keys else torch.zeros(0, dtype=torch.int64, device=self.device)
            vals = torch.cat(c._arb_vals) if c._arb_vals else \
                torch.zeros((0, self.ps_logic.dim), dtype=torch.float32, device=self.device)
            upd = ps.push_keys(keys, vals, lr=self.ps_logic.lr, return_updated=emit)
            for out in self.ps_logic.after_push(upd):
                self._emit(Right(out))

    def _push_rounds(self, plan, c) -> None:
        """``combine="sequential"``: the j-th push of a key in this micro-batch
        travels in round j, so a non-associative user rule sees the pushes one
        at a time in request order, as the reference's per-record PS applies
        them.  Rounds = the most repeats of a key on any rank (one host sync and
        a max all-reduce: the price of the exact order)."""
        U, D = plan.n_unique, self.ps_logic.dim
        dev = self.device
        if c._seq:
            pos = torch.cat([p for p, _, _ in c._seq])
            d = torch.cat([x.to(self.ps_logic.dtype) for _, x, _ in c._seq])
            m = torch.cat([torch.ones(p.numel(), dtype=torch.bool, device=dev) if mk is None else mk
                           for p, _, mk in c._seq])
        else:
            pos = torch.zeros(0, dtype=torch.int64, device=dev)
            d = torch.zeros((0, D), dtype=self.ps_logic.dtype, device=dev)
            m = torch.zeros(0, dtype=torch.bool, device=dev)
        pos = torch.where(m, pos, torch.full_like(pos, U))  # masked pushes sit out every round
        order = torch.argsort(pos, stable=True)
        sp = pos[order]
        first = torch.ones(sp.numel(), dtype=torch.bool, device=dev)
        first[1:] = sp[1:] != sp[:-1]
        idx = torch.arange(sp.numel(), device=dev)
        start = torch.cummax(torch.where(first, idx, torch.zeros_like(idx)), 0).values
        occ = torch.empty_like(idx)
        occ[order] = idx - start
        local = int(occ[pos < U].max()) + 1 if bool((pos < U).any()) else 0
        rounds = int(self.comm.max_over_ranks(float(local)))
        emit = self.ps_logic.emit == "push"
        for j in range(max(rounds, 1)):
            sel = (occ == j) & (pos < U)
            p = torch.where(sel, pos, torch.full_like(pos, U))
            buf = torch.zeros((U + 1, D), dtype=self.ps_logic.dtype, device=dev)
            buf[p] = d
            hit = torch.zeros(U + 1, dtype=torch.bool, device=dev)
            hit[p] = True
            updated = self.ps_logic.ps.push(plan, buf[:U], lr=self.ps_logic.lr, return_updated=emit, mask=hit[:U])
            self.counters.add("pushes", plan.n_unique)
            for out in self.ps_logic.after_push(updated):
                self._emit(Right(out))

    def _locked_step(self, keys, reqs, flag) -> None:
        """LockPSLogic semantics (``M/server/LockPSLogicA.scala:13-46``): a pulled key
        is held by one puller until its push; per round every key goes to its
        earliest pending request (lowest rank wins across workers), the others
        wait for a later round and then read the updated value.  Rounds repeat
        (collectively) until no rank has pending requests.  The worker sees each
        answered subset as a ``PulledBatch`` whose ``index`` lists the positions
        of the answered requests in its original ``pull``."""
        c = self.client
        lps = self.ps_logic.locked
        dim, op = self.ps_logic.dim, self.ps_logic.op
        n = keys.numel()
        req_of = torch.zeros(n, dtype=torch.int64, device=self.device)
        for i, r in enumerate(reqs):
            req_of[r.off:r.off + r.n] = i
        pending = torch.arange(n, device=self.device)
        while True:
            if pending.numel():  # the earliest pending request of every key
                uk, inv = torch.unique(keys[pending], return_inverse=True)
                cand = torch.full((uk.numel(),), n, dtype=torch.int64, device=self.device)
                cand.scatter_reduce_(0, inv, pending, reduce="amin")
                # torch.unique orders by key; the plan slots below are looked up by
                # request position (searchsorted), so order the candidates by position
                cand = cand.sort().values
            else:
                cand = pending
            pull = lps.acquire(keys[cand], flag=int(pending.numel() > 0))
            if not any(pull.plan.peer_flags):
                break
            plan, rows = pull.plan, pull.rows
            got = cand[pull.request_granted()]
            # holders that push nothing release the value unchanged
            new_vals = rows.float().clone() if op == "set" else \
                torch.zeros((plan.n_unique, dim), dtype=torch.float32, device=self.device)
            if got.numel():
                c._plan, c._acc, c._mask, c._direct = plan, None, None, None
                saved_pos = plan.pos
                for i, r in enumerate(reqs):
                    sel = got[req_of[got] == i]
                    if sel.numel() == 0:
                        continue
                    rpos = saved_pos[torch.searchsorted(cand, sel)]
                    c._req = _Request(keys[sel], r.payload, 0, sel.numel())
                    plan.pos = rpos  # push() maps this sub-request through plan.pos
                    self.worker_logic.on_pull_recv_batch(
                        PulledBatch(keys[sel], rows, rpos, r.payload, index=sel - r.off), c)
                plan.pos = saved_pos
                c._req = None
                if c._direct is not None:
                    new_vals = c._direct.float()
                elif c._acc is not None:
                    new_vals = torch.where(c._mask.view(-1, 1), c._acc, new_vals) if op == "set" else c._acc
                c._plan = None
            lps.release(pull, new_vals, mode=op)
            if self.ps_logic.emit == "push" and got.numel():
                g = plan.pos[torch.searchsorted(cand, got)].long()
                val = rows.float()[g] + new_vals[g] if op == "add" else new_vals[g]
                self._emit(Right((keys[got], val)))
            done = torch.zeros(n, dtype=torch.bool, device=self.device)
            done[got] = True
            pending = pending[~done[pending]]

    def finish(self) -> List[Any]:
        """Drain the pipeline, close the worker and the PS logic; returns the
        outputs collected on this rank (empty with an ``output_sink``)."""
        if self.pipe is not None:
            self.pipe.drain()
        if self.graphs is not None:  # no replays after the end: free the graphs now
            self.graphs.release()
        with stage("engine.close", self.timer):
            self.worker_logic.close(self.client)
            for out in self.ps_logic.close():
                self._emit(Right(out))
        close = getattr(self.output_sink, "close", None)
        if callable(close):
            close()
        return self.outputs

    def _run_phase(self, source: Iterable) -> None:
        it = iter(source)
        self.pipe.reset_flags()
        done = False
        while True:
            if not done:
                batch = next(it, _END)
                done = batch is _END
            self.submit(None if done else batch, flag=int(done))
            if self.pipe.all_flagged:
                break
        if self.pipe is not None:
            self.pipe.drain()

    def execute(self, source: Iterable, worker_logic: BatchedWorkerLogic, ps_logic: DevicePSLogic,
                model=None, worker_model=None) -> List[Any]:
        """Run a whole job on this rank: open, optional model load, every
        micro-batch of ``source`` (this rank's partition), end-of-input replay
        phases, close.  Returns this rank's outputs."""
        if ps_logic.locking:
            raise NotImplementedError("execute() with a locking PS logic: drive it with submit()/finish()")
        self.start(worker_logic, ps_logic)
        if self.comm.rank >= self.worker_parallelism:
            # no worker subtask on this rank: it serves its shard and joins the collectives.
            # Each rank passes its OWN input (SPMD), so data given here would be dropped --
            # the reference's workerParallelism spreads input over the worker subtasks
            # instead; the caller must partition it over ranks < worker_parallelism
            it = iter(source)
            if next(it, _END) is not _END:
                raise ValueError(f"rank {self.comm.rank} runs no worker (worker_parallelism="
                                 f"{self.worker_parallelism}) but was given input: partition the input over ranks "
                                 f"0..{self.worker_parallelism - 1}")
            source = ()
        if model is not None or worker_model is not None:
            self.load_model(model, worker_model)
        if self.iteration_wait_time is not None:
            source = idle_timeout(source, self.iteration_wait_time)
        self._run_phase(source)
        while True:  # on_eof replays (offline epochs) until every rank's worker is done
            more = self.worker_logic.on_eof(self.client)
            any_more = self.comm.sum_over_ranks(0.0 if more is None else 1.0) > 0
            if not any_more:
                break
            self._run_phase(more if more is not None else ())
        return self.finish()


_END = object()


def idle_timeout(source: Iterable, wait_ms: float) -> Iterator:
    """End ``source`` when no element arrived for ``wait_ms`` (``iterationWaitTime``,
    ``M/FlinkParameterServer.scala:49-52``; 0 = never).  A reader thread feeds a
    queue so a blocking source cannot hold the engine past the timeout."""
    if not wait_ms:
        yield from source
        return
    q: "queue.Queue" = queue.Queue(maxsize=64)

    def reader():
        try:
            for x in source:
                q.put(x)
        finally:
            q.put(_END)

    threading.Thread(target=reader, daemon=True).start()
    while True:
        try:
            x = q.get(timeout=wait_ms / 1000.0)
        except queue.Empty:
            return
        if x is _END:
            return
        yield x


def shard_batch(tensors: Sequence[torch.Tensor], key: torch.Tensor, rank: int, world: int):
    """Rows of ``tensors`` whose ``key % world == rank`` (``partitionCustom`` by key,
    e.g. ratings by ``user % W``, ``M/matrix/factorization/PSOnlineMatrixFactorization.scala:62-64``)."""
    m = (key.long().abs() % world) == rank
    return tuple(t[m] for t in tensors)


class FoldSink:
    """Output sink folding tensor outputs ``(ids, rows)`` last-writer-wins into
    dense device tables -- the model the reference's tests rebuild from the
    output stream (``T/matrix/factorization/PSOfflineMatrixFactorizationTest.scala:75-82``)."""

    def __init__(self, num_ids: int, dim: int, device="cpu", which: str = "both"):
        self.which = which
        self.tables = {k: torch.zeros((num_ids, dim), dtype=torch.float32, device=device) for k in ("left", "right")}
        self.seen = {k: torch.zeros(num_ids, dtype=torch.bool, device=device) for k in ("left", "right")}

    def __call__(self, e) -> None:
        side = "left" if isinstance(e, Left) else "right"
        if self.which not in ("both", side):
            return
        ids, rows = e.value
        ids = ids.long().to(self.tables[side].device)
        self.tables[side][ids] = rows.float().to(self.tables[side].device).reshape(ids.numel(), -1)
        self.seen[side][ids] = True

    def folded(self, side: str):
        """``{id: row}`` of one side (host numpy rows)."""
        idx = torch.nonzero(self.seen[side]).flatten()
        vals = self.tables[side][idx].cpu().double().numpy()
        return {int(i): vals[k] for k, i in enumerate(idx.tolist())}


def fold_outputs(outputs: Iterable) -> tuple:
    """``({worker id: row}, {ps id: row})`` from a list of tensor outputs, last
    writer wins (host dicts)."""
    res = ({}, {})
    for e in outputs:
        side = 0 if isinstance(e, Left) else 1
        ids, rows = e.value
        if ids.numel() == 0:
            continue
        rows = rows.detach().double().cpu().reshape(ids.numel(), -1).numpy()
        for k, i in enumerate(ids.reshape(-1).tolist()):
            res[side][int(i)] = rows[k]
    return res


def transform_tensor(source: Iterable, worker_logic: BatchedWorkerLogic, ps_logic: DevicePSLogic, *,
                     comm: Optional[Comm] = None, staleness: int = 0, iteration_wait_time: Optional[float] = None,
                     output_sink: Optional[Callable] = None, model=None, worker_model=None, graph: bool = False,
                     capacity: Optional[int] = None, worker_parallelism: Optional[int] = None,
                     ps_parallelism: Optional[int] = None) -> List[Any]:
    """Tensor-engine ``transform`` on this rank (SPMD under torchrun): ``source``
    is this rank's iterable of micro-batches.  ``graph`` / ``capacity``: captured
    steps / fixed-shape plans; ``worker_parallelism`` / ``ps_parallelism``: at most
    the world each (``TensorRuntime``)."""
    rt = TensorRuntime(comm, staleness, iteration_wait_time, output_sink, graph=graph, capacity=capacity,
                       worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism)
    return rt.execute(source, worker_logic, ps_logic, model=model, worker_model=worker_model)


def transform_tensor_with_model_load(model, source, worker_logic, ps_logic, **kw) -> List[Any]:
    """``transformWithModelLoad`` on the tensor engine: ``model`` = this rank's
    ``(id, value)`` records for the PS."""
    return transform_tensor(source, worker_logic, ps_logic, model=model, **kw)


def transform_tensor_with_double_model_load(model, source, worker_logic, ps_logic, **kw) -> List[Any]:
    """``transformWithDoubleModelLoad``: ``model`` = this rank's ``Left((id, v))``
    (PS) / ``Right((id, v))`` (worker-resident) records, or a pair
    ``(ps_records, worker_records)``."""
    if isinstance(model, tuple) and len(model) == 2 and not isinstance(model[0], (Left, Right)):
        ps_recs, w_recs = model
    else:
        recs = list(model)
        ps_recs = [tuple(e.value) for e in recs if isinstance(e, Left)]
        w_recs = [tuple(e.value) for e in recs if isinstance(e, Right)]
    return transform_tensor(source, worker_logic, ps_logic, model=ps_recs, worker_model=w_recs, **kw)
