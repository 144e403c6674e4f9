"""The tensor-path parameter server: batched pull / push over RCCL all-to-all.

Replaces the reference's per-record Flink iteration
(``M/FlinkParameterServer.scala:215-335``) with a micro-batch protocol:

``plan_begin(keys)`` (stage A, nothing blocks the host)
    1. de-duplicate the batch's keys and group them by owning shard (K1,
       ``ops.DedupWorkspace``) -- the batch's own pre-reduction, the GPU
       analogue of the combining senders (``M/common/CombinationLogic.scala``);
    2. exchange per-shard counts (tiny all-to-all, one ``(count, flag)`` pair
       per peer: the flag carries "this rank's input is exhausted", so the
       end-of-input barrier of ``FlinkEOF`` rides on the same message);
    3. copy the counts into pinned host memory (non-blocking) and record an
       event.
``plan_end(pending)`` (stage B)
    4. wait for that event -- recorded one micro-batch earlier in a pipelined
       loop, so in steady state it has long completed: the host never stalls
       the device on split sizes (torch needs them on the host);
    5. X1: all-to-all of the unique local keys to their owners.
``pull``: 6. owners gather their rows (K2) into the wire dtype;
    7. X2: all-to-all of the rows back.  Rows return in request order, so
       ``rows[pos[b]]`` is request ``b``'s parameter (positional FIFO).
``push(plan, deltas)``
    8. X1': all-to-all of per-unique-key deltas (pre-reduced on the worker) to
       the owners;
    9. owners apply them (K3: add / set / sgd / adagrad / add_renorm).

``world == 1`` keeps the same code path with local copies instead of RCCL.

Fixed-shape plans (``TensorPS.capacity``): every rank sends every peer exactly
``C`` key slots per micro-batch with its (count, flag) in a two-int header --
one all-to-all of ``[W, C + 2]`` int32 replaces the count exchange, its host copy
and the key all-to-all; padding slots carry key -1 (served as zero rows, skipped
by the apply).  No split size is ever needed on the host, so a micro-batch step
has fixed shapes and can be captured with its RCCL collectives into a hipGraph
(``core.step_graph``); peers' end-of-input flags reach the host one micro-batch
later (``BoundedStalenessPipeline.poll_flags``).
Staleness: every request in a micro-batch reads the table as of step 6;
``parallel.staleness.BoundedStalenessPipeline`` orders the stages of several
micro-batches so pull ``k`` is served before the pushes of ``k-s .. k-1``
(``max_inflight``), the bounded-staleness analogue of ``pullLimit``
(``M/WorkerLogic.scala:176-225``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from .. import ops
from ..api.batched import MaskedPair
from ..utils.tracing import stage
from .comm import Comm
from .table import ShardedTable


@dataclass
class PullPlan:
    send_splits: List[int]   # unique keys this worker sends to each shard
    recv_splits: List[int]   # keys each worker sends to this shard
    recv_keys: torch.Tensor  # local keys this shard must serve / apply
    pos: torch.Tensor        # request -> row of the pulled/delta buffers
    n_unique: int
    peer_flags: List[int] = field(default_factory=list)  # flag each rank sent with this plan
    n_requests: int = 0
    recv_rows: Optional[torch.Tensor] = None  # rows of recv_keys in the shard (cached by serve)
    #: static plans (world 1): n_unique is an upper bound; valid[j] marks the real unique keys
    valid: Optional[torch.Tensor] = None
    #: identity plan (world 1, a batch at least as large as the key space): the unique
    #: keys are the whole key space in order, so ``pos`` is the key itself
    identity: bool = False
    #: False: a request plan (no de-duplication) -- keys may repeat, so pushes apply
    #: with atomics instead of the unique-key read-modify-write
    unique: bool = True
    ready: Optional[object] = None  # event to wait for before the plan's device data is read
    #: every peer's segment of ``recv_keys`` holds distinct keys (each peer chose a
    #: de-duplicating plan; ranks choose per batch size, so a small batch on one rank
    #: may arrive as a request plan at owners whose own plan de-duplicates)
    recv_unique: bool = True
    #: fixed-shape plan: the peers' flags stay on the device (``[W]`` int32)
    flags_dev: Optional[torch.Tensor] = None
    fixed: bool = False
    #: the serve handed out the shard itself (``zero_copy_identity``), not a snapshot
    zero_copy: bool = False
    #: static plans: ``valid.sum()`` on the device (counted once for pulls and pushes)
    n_valid: Optional[torch.Tensor] = None
    #: static dense plans: ``recv_keys`` with -1 on the padding slots (the rows a push
    #: applies), built with the plan instead of per push
    push_rows: Optional[torch.Tensor] = None
    #: owner stream (``TensorPS.owner_stream``): the key all-to-all's work -- the serve
    #: waits for it on the owner stream instead of the compute stream
    key_work: Optional[object] = None


@dataclass
class PendingPlan:
    """A plan after stage A: device-side dedup done, counts on their way to the host."""
    n: int
    counts: torch.Tensor     # int32[W] unique keys per owner (own copy)
    uniq: torch.Tensor       # int32[>= U] unique local keys grouped by owner
    pos: torch.Tensor        # int32[n]
    host: torch.Tensor       # int32[W, 4]: (sent count, sent flag, recv count, recv flag) per peer;
                             # world 1: int32[1], the count alone (the flag never leaves the rank)
    event: Optional[object]  # torch.cuda.Event or None (host tensors: already complete)
    flag: int = 0
    valid: Optional[torch.Tensor] = None  # static plan: [n_bound] bool
    n_bound: int = 0
    identity: bool = False
    unique: bool = True
    static: bool = False  # sizes known on the host (world 1): nothing to wait for
    ready: Optional[object] = None  # event the plan's inputs (a presence hint) are ready behind
    #: ``TensorPS._plan_seq`` when the counts' event was recorded
    seq: int = 0
    #: columns of ``host`` holding (sent count, sent flag, recv count, recv flag): several
    #: tables planned together (``plan_begin_multi``) share one exchange and one host copy
    cols: tuple = (0, 1, 2, 3)
    #: fixed-shape plan: the received ``[W, C + 2]`` header + key slots
    fixed: Optional[torch.Tensor] = None
    push_rows: Optional[torch.Tensor] = None  # static dense plan: recv keys, -1 on the padding



@dataclass
class PendingPush:
    """A push whose all-to-all is posted, not yet applied (``TensorPS.push(defer=True)``)."""
    plan: PullPlan
    recv: torch.Tensor
    work: Optional[object]
    opt: str
    lr: float


class _EventWork:
    """A ``Work``-like handle over a device event: ``wait()`` orders the caller's stream."""

    def __init__(self, event):
        self.event = event

    def wait(self) -> None:
        torch.cuda.current_stream().wait_event(self.event)

    def is_completed(self) -> bool:
        return self.event.query()


class TensorPS:
    def __init__(self, table: ShardedTable, comm: Comm, wire_dtype=torch.float32):
        self.table = table
        self.comm = comm
        self.wire_dtype = wire_dtype
        # sparse-id tables (parallel.hash_table) dedup through the per-batch hashed claim map
        #: PS shards (``ps_parallelism``): shard s lives on rank s; ranks >= shards hold
        #: none and receive no keys.  The owner of a key is computed on the device from
        #: the table's partition over ``shards`` (``|id| % P`` or ``|id| // ceil(F/P)``)
        self.shards = int(getattr(table, "world", comm.world))
        if self.shards > comm.world or self.shards < 1:
            raise ValueError(f"{self.shards} PS shards on {comm.world} ranks: need 1 <= shards <= ranks")
        if self.shards != comm.world and getattr(table, "sparse", False):
            raise ValueError("sparse (hash-table) shards need one shard per rank")
        self.dedup = ops.DedupWorkspace(table.key_space, self.shards, table.part_kind, table.block, table.device,
                                        hashed=True if getattr(table, "sparse", False) else None,
                                        out_world=comm.world)
        self._stats = {"pulls": 0, "unique": 0, "steps": 0, "host_waits": 0, "host_stalls": 0, "pushes": 0}
        #: plans whose counts went to the host through an event (``PendingPlan.seq``)
        self._plan_seq = 0
        #: static plans pad their unique keys to a bound: the exact counts accumulate on
        #: the device (no per-step sync) and are folded in when ``stats`` is read
        self._lazy: dict = {}
        self.timer = None  # utils.metrics.StageTimer (optional)
        #: pushes carry a validity column (set by the device PS logic on every rank
        #: alike): rows a worker did not push are skipped by the apply and by the
        #: per-push output instead of being applied as zero deltas
        self.masked_push = False
        self._pinned = table.device.type == "cuda"
        #: world 1, dense shard: plans whose sizes need no device->host copy -- the
        #: unique keys are padded to ``min(n, key space)`` rows (padding gathers row 0
        #: and is never applied), so a micro-batch issues no host sync at all
        self.static = False
        self._iota: Optional[torch.Tensor] = None
        #: de-duplicate each micro-batch's keys (True), ship every request (False: a
        #: request plan), or decide per batch size (None): requests go undeduplicated
        #: when the key space is at least ``REQUEST_PLAN_RATIO`` times the batch (repeats
        #: are then rare, so the dedup pass costs more than the rows it saves: PA over 1B
        #: features repeats ~8 % of 4M keys) and the rule is additive (atomic apply)
        self.dedup_mode: Optional[bool] = None
        self._req_iota: Optional[torch.Tensor] = None
        #: static request / identity plans reference the caller's key tensor (``uniq`` /
        #: ``pos`` = the keys) until the batch is served and pushed, which with a
        #: pipeline is one or more submits later: they keep a copy unless the owner
        #: guarantees its key tensors are never rewritten (``keys_stable``)
        self.keys_stable = False
        #: world-1 identity plans serve the shard itself instead of a copy (the pulled
        #: rows are the table): for owners whose workers only READ the pulled rows and
        #: accept reading them fresher than served (never staler: the bound still holds)
        self.zero_copy_identity = False
        #: fixed-shape plans (module docstring): the most keys a rank plans per
        #: micro-batch.  ``C`` = this capacity for request plans, capped at the largest
        #: shard for de-duplicating ones; the plan kind is chosen from the capacity, so
        #: every rank picks the same.  Each exchange then moves ``W * C`` rows instead of
        #: the unique keys: for the small, host-bound micro-batches.  Used by
        #: ``plan_begin`` (the pipelined path); ``plan()`` keeps dynamic plans.
        self.capacity: Optional[int] = None
        self._slots: Optional[torch.Tensor] = None
        #: the OWNER side on its own stream (``BoundedStalenessPipeline(owner_stream=True)``
        #: at world > 1 on the GPU): the serve of a pull and the apply of a push run there,
        #: each after its all-to-all, so the compute stream never waits for a key or push
        #: transfer -- only for the answer rows it is about to compute on.  Every
        #: all-to-all (and the count exchange) is posted asynchronously; the counts reach
        #: the host through ``_aux_stream``.  Stream order on the owner stream keeps the
        #: staleness bound (serve k is enqueued after apply k - s - 1, as before).
        self.owner_stream = None
        self._aux_stream = None
        self._compute_stream = None
        #: the exchanges are posted asynchronously on ONE stream (``BoundedStalenessPipeline``'s
        #: interleaved schedule): the key all-to-all's work is waited for right before the
        #: serve and a deferred push (``push(defer=True)``) right before its apply, so the
        #: transfers overlap the compute enqueued in between without a second stream
        self.async_exchange = False
        #: set by the pipeline around a compute that pushes through the engine: deferrable
        #: pushes are posted and appended here as ``(self, PendingPush)`` instead of applied
        self._defer_into: Optional[list] = None

    @property
    def stats(self) -> dict:
        """pulls = requests, unique = unique keys planned (exact also for padded static
        plans), steps = plans, pushes = unique keys applied; host_waits = ``plan_end``
        calls that found their counts not yet on the host (the host waited: with a
        device-bound pipeline that is plain back-pressure), host_stalls = the subset
        where nothing had been enqueued after those counts -- the device drains and
        idles while the host waits (``plan()`` back to back, or a pipeline without
        lookahead)."""
        if self._lazy:
            for k, parts in self._lazy.items():
                self._stats[k] += int(torch.stack(parts).sum().item())
            self._lazy = {}
        return self._stats

    #: per-step device counts stay 0-dim tensors (no accumulate kernel per step), folded
    #: into one every ``_LAZY_FOLD`` steps
    _LAZY_FOLD = 256

    def _count_lazy(self, key: str, valid: torch.Tensor, bound: Optional[int] = None,
                    total: Optional[torch.Tensor] = None):
        """Add ``valid.sum()`` (or the precomputed ``total``) to ``stats[key]`` without a
        host sync; returns the device count (None while a graph is captured)."""
        if valid.is_cuda and torch.cuda.is_current_stream_capturing():
            # a captured step (core.step_graph) replays its host-side increments: count the
            # bound there (a device counter inside the graph would not be read per replay)
            self._stats[key] += valid.numel() if bound is None else bound
            return None
        n = valid.sum() if total is None else total
        parts = self._lazy.setdefault(key, [])
        parts.append(n)
        if len(parts) >= self._LAZY_FOLD:
            self._lazy[key] = [torch.stack(parts).sum()]
        return n

    #: key space / batch ratio above which ``dedup_mode = None`` ships requests undeduplicated
    REQUEST_PLAN_RATIO = 64

    def dedups(self, n: int) -> bool:
        """Does a micro-batch of ``n`` requests get a de-duplicating plan?"""
        if self.dedup_mode is not None:
            return bool(self.dedup_mode) or not self._request_plans_ok()
        return not (self._request_plans_ok() and n > 0 and int(self.table.key_space) >= self.REQUEST_PLAN_RATIO * n)

    def _request_plans_ok(self) -> bool:
        """Request plans need an additive rule (repeated keys apply atomically) and a
        dense shard (the sparse hash shard and lookup partitions resolve keys once)."""
        return (getattr(self.table, "optimizer", "") in ("add", "sgd") and not self.masked_push
                and not getattr(self.table, "sparse", False) and getattr(self.table, "partition", "") != "lookup")

    def identity_for(self, n: int) -> bool:
        """Will a static plan of ``n`` requests be the identity plan?  (World 1, a
        dense shard and ``n >= key space``: instead of de-duplicating, the plan takes
        the whole key space in order -- ``pos`` = the key, a presence flag per key --
        so a worker may bucket its requests by key before the plan exists.)"""
        return (self.static and self.comm.world == 1 and not getattr(self.table, "sparse", False)
                and getattr(self.table, "partition", "") != "lookup" and n >= int(self.table.key_space))

    def fixed(self) -> bool:
        """Does ``plan_begin`` make fixed-shape plans?"""
        return self.capacity is not None and not self.static and not getattr(self.table, "sparse", False)

    def fixed_slots(self, unique: bool) -> int:
        """``C``: key slots per peer of a fixed-shape plan (the same on every rank)."""
        C = int(self.capacity)
        if unique:  # de-duplicated keys to one owner: at most its shard's rows
            t = self.table
            C = min(C, max(t.part.shard_size(t.num_ids, r) for r in range(self.shards)))
        return max(C, 1)

    def _fixed_plan(self, keys: torch.Tensor, flag: int, dedup: Optional[bool]) -> PendingPlan:
        """Stage A of a fixed-shape plan: dedup (or route), slot layout, and the one
        ``[W, C + 2]`` all-to-all of (count, flag, keys) -- no host copy."""
        n = keys.numel()
        if n > self.capacity:
            raise ValueError(f"fixed-shape plans: {n} keys in a micro-batch, capacity {self.capacity}")
        W = self.comm.world
        unique = bool(dedup) or self.dedups(int(self.capacity))  # from the capacity: every rank alike
        C = self.fixed_slots(unique)
        with stage("ps.dedup" if unique else "ps.route", self.timer):
            counts, prefix, uniq, pos = self.dedup.run(keys) if unique else self.dedup.route(keys)
        dev = keys.device
        if self._slots is None or self._slots.numel() != C or self._slots.device != dev:
            self._slots = torch.arange(C, dtype=torch.int64, device=dev)
        j = self._slots.view(1, C)
        start = prefix[:W].to(torch.int64).view(W, 1)
        valid = j < counts[:W].to(torch.int64).view(W, 1)
        if uniq.numel() == 0:
            uniq = torch.full((1,), -1, dtype=torch.int32, device=dev)
        idx = (start + j).clamp_max(uniq.numel() - 1)
        send = torch.empty((W, C + 2), dtype=torch.int32, device=dev)
        send[:, 0] = counts[:W]
        send[:, 1] = int(flag)
        send[:, 2:] = torch.where(valid, uniq[idx], torch.full_like(idx, -1, dtype=torch.int32))
        # request b -> slot of its key: owner segment * C + rank inside the owner's group
        u = pos.to(torch.int64)
        owner = torch.searchsorted(prefix[1:W + 1].to(torch.int64).contiguous(), u, right=True)
        slot = (owner * C + (u - start.view(W)[owner])).to(torch.int32)
        if self.dedup.clear_after:
            self.dedup.reset_claims(keys)
        with stage("ps.key-a2a", self.timer):
            recv = self.comm.all_to_all(send.view(-1), [C + 2] * W, [C + 2] * W).view(W, C + 2)
        self._count_lazy("unique", counts[:W], bound=n)
        return PendingPlan(n, counts, None, slot, None, None, int(flag), n_bound=W * C, unique=unique, static=True,
                           fixed=recv)

    # ----------------------------------------------------------------- planning
    def plan_begin(self, keys: torch.Tensor, flag: int = 0, dedup: Optional[bool] = None,
                   presence=None, fixed: bool = True) -> PendingPlan:
        """Stage A: dedup + count exchange, counts copied to pinned host memory
        asynchronously.  Collective: every rank calls it once per micro-batch
        (with empty ``keys`` when it has nothing to pull).  ``flag`` (an int) is
        delivered to every peer with the counts (``PullPlan.peer_flags``).  ``dedup``:
        force (True) the de-duplicating plan instead of ``dedups(n)``'s choice.
        ``presence``: ``(uint8 flags [key space], event)`` of the keys, computed by the
        caller (an identity plan then skips its marking pass; other plans ignore it).
        ``fixed = False``: a dynamic plan even with a ``capacity`` set."""
        a = self._stage_a(keys, flag, dedup, presence, fixed)
        if isinstance(a, PendingPlan):
            return a
        return self._pending(*a, flag=flag)

    def _stage_a(self, keys: torch.Tensor, flag: int = 0, dedup: Optional[bool] = None, presence=None,
                 fixed: bool = True):
        """The device part of stage A: a finished (static) ``PendingPlan``, or
        ``(n, counts, uniq, pos, unique)`` still needing the count exchange."""
        keys = self.table.route_keys(keys.to(device=self.table.device)).to(torch.int32).contiguous()
        n = keys.numel()
        if fixed and self.fixed():
            return self._fixed_plan(keys, flag, dedup)
        if self.identity_for(n):
            ks = int(self.table.key_space)
            if self._iota is None or self._iota.numel() != ks:
                self._iota = torch.arange(ks, dtype=torch.int32, device=keys.device)
            ready = None
            if presence is not None and presence[0].numel() == ks:
                present, ready = presence  # the caller's flags (e.g. from its partition pass)
            else:
                with stage("ps.presence", self.timer):
                    present = torch.zeros(ks, dtype=torch.uint8, device=keys.device)
                    ops.mark_rows(present, keys)
            if not self.keys_stable:
                keys = keys.clone()
            return PendingPlan(n, None, self._iota, keys, None, None, int(flag), valid=present.view(torch.bool),
                               n_bound=ks, identity=True, static=True, ready=ready)
        W = self.comm.world
        if not (dedup or self.dedups(n)):
            if W == 1 and self.static:  # every request is its own row: nothing to compute
                if self._req_iota is None or self._req_iota.numel() < n:
                    self._req_iota = torch.arange(max(n, 1), dtype=torch.int32, device=keys.device)
                return PendingPlan(n, None, keys if self.keys_stable else keys.clone(), self._req_iota[:n], None,
                                   None, int(flag), n_bound=n,
                                   unique=False, static=True)
            with stage("ps.route", self.timer):
                counts, prefix, uniq, pos = self.dedup.route(keys, fresh=True)
            return n, counts, uniq, pos, False
        static1 = W == 1 and self.static and not getattr(self.table, "sparse", False)
        with stage("ps.dedup", self.timer):
            # a dynamic plan keeps its outputs across later plans: fresh tensors, no copy
            counts, prefix, uniq, pos = self.dedup.run(keys, fresh=not static1)
        if static1:
            nb = min(n, int(self.table.key_space))
            # padding slot j serves the real key uniq[j mod U]: real rows only (the
            # close-time dump stays exact) and spread over all of them (a single padding
            # row shared by millions of slots serialised the gather on one cache line)
            gkeys, valid, pos_c, push_rows = ops.static_plan(uniq, prefix, nb, pos)
            if self.dedup.clear_after:
                self.dedup.reset_claims(gkeys)
            return PendingPlan(n, counts, gkeys, pos_c, None, None, int(flag), valid=valid, n_bound=nb,
                               static=True, push_rows=push_rows)
        return n, counts, uniq, pos, True

    def _own(self, t: torch.Tensor) -> torch.Tensor:
        """``t``, cloned if it lives in the dedup workspace (reused by the next plan)."""
        ws = self.dedup
        p = t.untyped_storage().data_ptr()
        for a in ("counts", "prefix", "uniq", "pos"):
            w = getattr(ws, a, None)
            if w is not None and w.untyped_storage().data_ptr() == p:
                return t.clone()
        return t

    @staticmethod
    def _wire_counts(counts: torch.Tensor, W: int, unique: bool) -> torch.Tensor:
        """Per-peer counts as sent in the count exchange: ``2 * count + 1`` for a
        request plan, so an owner knows which segments may repeat keys."""
        return counts.view(W, 1).to(torch.int32) * 2 + (0 if unique else 1)

    def _pending(self, n, counts, uniq, pos, unique: bool = True, flag: int = 0) -> PendingPlan:
        """Stage A's count exchange of a computed (de-duplicated or request) plan."""
        W = self.comm.world
        # the workspace is reused by the next plan_begin: this plan keeps copies of what
        # lives there (a fresh-output dedup / the CPU twins return tensors of their own)
        counts = self._own(counts)
        uniq = self._own(uniq[:n])
        pos = self._own(pos)
        if W == 1:  # no peers: only the count travels (device -> host), no exchange / packing ops
            if self._pinned:
                host = torch.empty(1, dtype=torch.int32, pin_memory=True)
                host.copy_(counts[:1].to(torch.int32), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            else:
                host, ev = counts[:1].to("cpu", torch.int32), None
            self._plan_seq += 1
            return PendingPlan(n, counts, uniq, pos, host, ev, int(flag), unique=unique, seq=self._plan_seq)
        send = ops.pack_counts(counts, W, not unique, flag)  # [W, 2]: 2 count + request, flag
        if (self.owner_stream is not None or self.async_exchange) and self._pinned:
            host, ev = self._counts_async(send)
        else:
            with stage("ps.count-a2a", self.timer):
                recv = self.comm.exchange_counts(send)
            both = torch.cat([send, recv.to(send.device)], dim=1)  # [W, 4]
            if self._pinned:
                host = torch.empty((W, 4), dtype=torch.int32, pin_memory=True)
                host.copy_(both, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            else:
                host, ev = both.to("cpu"), None
        self._plan_seq += 1
        return PendingPlan(n, counts, uniq, pos, host, ev, int(flag), unique=unique, seq=self._plan_seq)

    def _counts_async(self, send: torch.Tensor):
        """Owner-stream mode: the count exchange posted asynchronously; the pinned host
        copy of ``[send | recv]`` runs on the aux stream behind it (a synchronous
        exchange would make the compute stream wait for every row transfer queued on the
        communicator before it).  Returns ``(pinned host tensor, event)``."""
        with stage("ps.count-a2a", self.timer):
            recv, work = self.comm.exchange_counts_async(send)
        host = torch.empty((send.shape[0], 2 * send.shape[1]), dtype=torch.int32, pin_memory=True)
        if work is None:  # the counts are already on this stream (no transfer in flight): copy here
            host.copy_(torch.cat([send, recv], dim=1), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            return host, ev
        cur = torch.cuda.current_stream(send.device)
        if self._aux_stream is None:
            self._aux_stream = torch.cuda.Stream(send.device)
        aux = self._aux_stream
        with torch.cuda.stream(aux):
            aux.wait_stream(cur)  # send was written on the compute stream
            work.wait()
            send.record_stream(aux)
            recv.record_stream(aux)
            host.copy_(torch.cat([send, recv], dim=1), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(aux)
        return host, ev

    def plan_end(self, pp: PendingPlan) -> PullPlan:
        """Stage B: split sizes from the host copy, key all-to-all."""
        if pp.fixed is not None:  # fixed-shape plan: the keys arrived in stage A
            W, C = pp.fixed.shape[0], pp.fixed.shape[1] - 2
            self._stats["pulls"] += pp.n
            self._stats["steps"] += 1
            return PullPlan([C] * W, [C] * W, pp.fixed[:, 2:].reshape(-1), pp.pos, W * C, [], pp.n,
                            unique=pp.unique, recv_unique=pp.unique, flags_dev=pp.fixed[:, 1], fixed=True)
        if pp.static:  # static world-1 plan: sizes known on the host, nothing to wait for
            if pp.ready is not None and self.table.device.type == "cuda":
                torch.cuda.current_stream(self.table.device).wait_event(pp.ready)
            self._stats["pulls"] += pp.n
            n_valid = None
            if pp.valid is not None:
                n_valid = self._count_lazy("unique", pp.valid)
            else:
                self._stats["unique"] += pp.n_bound
            self._stats["steps"] += 1
            return PullPlan([pp.n_bound], [pp.n_bound], pp.uniq, pp.pos, pp.n_bound, [pp.flag], pp.n,
                            valid=pp.valid, identity=pp.identity, unique=pp.unique, ready=pp.ready,
                            n_valid=n_valid, push_rows=pp.push_rows)
        if pp.event is not None:
            if not pp.event.query():
                self._stats["host_waits"] += 1
                if pp.seq == self._plan_seq:  # no later plan was enqueued behind these counts
                    self._stats["host_stalls"] += 1
            pp.event.synchronize()
        sc, _, rc, rf = pp.cols
        recv_unique = pp.unique
        if pp.host.dim() == 1:  # world 1
            c = int(pp.host[sc])
            send_splits, recv_splits, peer_flags = [c], [c], [pp.flag]
        else:  # counts travel as 2 * count + (request plan)
            h = pp.host.tolist()
            send_splits = [int(r[sc]) >> 1 for r in h]
            recv_splits = [int(r[rc]) >> 1 for r in h]
            recv_unique = not any(int(r[rc]) & 1 for r in h)
            peer_flags = [int(r[rf]) for r in h]
        n_unique = int(sum(send_splits))
        kw = None
        with stage("ps.key-a2a", self.timer):
            if self.owner_stream is not None or self.async_exchange:  # the serve waits for the keys
                recv_keys, kw = self.comm.all_to_all_async(pp.uniq[:n_unique], send_splits, recv_splits)
            else:
                recv_keys = self.comm.all_to_all(pp.uniq[:n_unique], send_splits, recv_splits)
        self._stats["pulls"] += pp.n
        self._stats["unique"] += n_unique
        self._stats["steps"] += 1
        return PullPlan(send_splits, recv_splits, recv_keys, pp.pos, n_unique, peer_flags, pp.n, unique=pp.unique,
                        recv_unique=recv_unique, key_work=kw)

    @staticmethod
    def plan_begin_multi(pss: Sequence["TensorPS"], keys_list: Sequence[torch.Tensor], flag: int = 0,
                         dedup: Optional[bool] = None) -> List[PendingPlan]:
        """Stage A of one micro-batch's plans on several tables (same ranks and
        device) with ONE count exchange and ONE device->host copy: the counts of
        every table and the flag travel as the columns of one ``[W, T + 1]``
        message (SGNS pulls from two tables per micro-batch: two exchanges and two
        host copies otherwise)."""
        if len(pss) != len(keys_list):
            raise ValueError("one key tensor per table")
        staged = [ps._stage_a(k, flag, dedup) for ps, k in zip(pss, keys_list)]
        comm = pss[0].comm
        dyn = [j for j, a in enumerate(staged) if not isinstance(a, PendingPlan)]
        out: List[PendingPlan] = [a if isinstance(a, PendingPlan) else None for a in staged]
        if not dyn:
            return out
        T, W = len(dyn), comm.world
        dev = staged[dyn[0]][1].device
        counts = [pss[j]._own(staged[j][1]) for j in dyn]  # the workspaces are reused by the next plan
        if W == 1:
            send = torch.cat([c[:1].to(torch.int32) for c in counts])  # [T]
            both = send
        else:
            cols = [TensorPS._wire_counts(c, W, staged[j][4]) for c, j in zip(counts, dyn)]
            cols.append(torch.full((W, 1), int(flag), dtype=torch.int32, device=dev))
            send = torch.cat(cols, dim=1).contiguous()  # [W, T + 1]
            if (pss[0].owner_stream is not None or pss[0].async_exchange) and dev.type == "cuda":
                both = None
                host, ev = pss[0]._counts_async(send)
            else:
                with stage("ps.count-a2a", pss[0].timer):
                    recv = comm.exchange_counts(send)
                both = torch.cat([send, recv.to(send.device)], dim=1)  # [W, 2T + 2]
        if both is None:
            pass
        elif dev.type == "cuda":
            host = torch.empty(tuple(both.shape), dtype=torch.int32, pin_memory=True)
            host.copy_(both, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = both.to("cpu"), None
        for t, j in enumerate(dyn):
            n, _, uniq, pos, unique = staged[j]
            cols = (t, T, t, T) if W == 1 else (t, T, T + 1 + t, 2 * T + 1)
            pss[j]._plan_seq += 1
            out[j] = PendingPlan(n, counts[t], pss[j]._own(uniq[:n]), pss[j]._own(pos), host, ev, int(flag), unique=unique,
                                 cols=cols, seq=pss[j]._plan_seq)
        return out

    def plan(self, keys: torch.Tensor, persistent: bool = False, flag: int = 0,
             dedup: Optional[bool] = None) -> PullPlan:
        """Stages A + B back to back (the host waits on this micro-batch's counts).
        Plans never alias the dedup workspace, so ``persistent`` is implied."""
        return self.plan_end(self.plan_begin(keys, flag, dedup, fixed=False))

    # --------------------------------------------------------------------- pull
    def serve(self, plan: PullPlan) -> torch.Tensor:
        with stage("ps.serve", self.timer):
            if plan.recv_rows is None:  # dense shards: the local key is the row; sparse: lookup-or-insert
                plan.recv_rows = self.table.rows_for(plan.recv_keys)[0]
            touched = getattr(self.table, "touched", None)
            sentinel = getattr(self.table, "sentinel", False)
            if not plan.identity or (touched is None and not sentinel):
                return self.table.serve_rows(plan.recv_rows, self.wire_dtype)
            # identity plan: every row is served, only the keys present count as pulled
            if self.zero_copy_identity and self.wire_dtype == self.table.weight.dtype:
                out = self.table.weight  # the pulled rows ARE the shard (read-only consumer)
                plan.zero_copy = True
            else:
                out = self.table.serve_rows(plan.recv_rows, self.wire_dtype, mark=False)
            if sentinel:  # flip the untouched sentinel of the present rows only
                ops.flip_masked(self.table.weight, plan.valid)
            else:
                touched |= plan.valid.view(torch.uint8)
            return out

    def _owner_enter(self, work, *tensors) -> None:
        """On the owner stream (current): order it after ``work`` (an all-to-all whose
        output it is about to read) or, without one, after the compute stream; keep the
        ``tensors`` (allocated on the compute stream) alive for its reads."""
        O = self.owner_stream
        if work is not None:
            work.wait()
        else:
            O.wait_stream(self._compute_stream)
        for t in tensors:
            if t is not None and t.is_cuda:
                t.record_stream(O)

    def owner_sync(self) -> None:
        """The compute stream waits for every serve / apply enqueued on the owner stream
        (end of a pipeline drain: the caller then reads the table)."""
        if self.owner_stream is not None:
            torch.cuda.current_stream(self.table.device).wait_stream(self.owner_stream)

    def pull_planned(self, plan: PullPlan, async_op: bool = False):
        """Serve + answer all-to-all of a planned pull: ``rows`` or ``(rows, work)``.
        Owner-stream mode (``async_op``): both run on the owner stream."""
        if async_op and self.owner_stream is not None:
            self._compute_stream = torch.cuda.current_stream(self.table.device)
            with torch.cuda.stream(self.owner_stream):
                self._owner_enter(plan.key_work, plan.recv_keys, plan.valid, plan.push_rows)
                plan.key_work = None
                served = self.serve(plan)
                with stage("ps.answer-a2a", self.timer):
                    rows, work = self.comm.all_to_all_async(served, plan.recv_splits, plan.send_splits)
                if work is None:  # no transfer (world 1): the compute stream waits for the serve
                    ev = torch.cuda.Event()
                    ev.record(self.owner_stream)
                    work = _EventWork(ev)
            return rows, work
        self.owner_sync()  # a serve on the compute stream: after every owner-stream apply
        if plan.key_work is not None:  # keys of an owner-stream plan served here instead
            plan.key_work.wait()
            plan.key_work = None
        served = self.serve(plan)
        with stage("ps.answer-a2a", self.timer):
            if async_op:
                return self.comm.all_to_all_async(served, plan.recv_splits, plan.send_splits)
            return self.comm.all_to_all(served, plan.recv_splits, plan.send_splits)

    def pull(self, keys: torch.Tensor):
        """Returns ``(rows[U, D] in wire dtype, plan)``; request b's row is ``rows[plan.pos[b]]``."""
        plan = self.plan(keys)
        return self.pull_planned(plan), plan

    def pull_async(self, keys: torch.Tensor):
        """Start a pull whose row all-to-all runs on the communicator's stream while
        the caller keeps computing; returns ``(rows, work, plan)`` -- wait on
        ``work`` (if not None) before reading ``rows``."""
        plan = self.plan(keys)
        rows, work = self.pull_planned(plan, async_op=True)
        return rows, work, plan

    # --------------------------------------------------------------------- push
    def push(self, plan: PullPlan, deltas: torch.Tensor, lr: float = 0.0, op: Optional[str] = None,
             return_updated: bool = False, mask: Optional[torch.Tensor] = None, defer: bool = False):
        """Send per-unique-key deltas ``[U, D]`` (fp32) to their owners and apply
        with ``op`` (default: the table's rule).  ``return_updated``: also return
        ``(global ids, new rows)`` of the keys applied on THIS shard -- the
        per-push ``(id, value)`` output of ``SimplePSLogic``
        (``M/server/SimplePSLogic.scala:24``).  ``mask[U]`` (bool) marks the keys
        actually pushed; it travels only when ``masked_push`` is set.  ``defer``: post the
        all-to-all and return a ``PendingPush`` -- ``apply_pending`` waits for it and
        applies (None when the push had to complete here)."""
        D = self.table.dim
        deltas = deltas.reshape(plan.n_unique, D)
        if self.masked_push:
            m = torch.ones(plan.n_unique, 1, dtype=deltas.dtype, device=deltas.device) if mask is None else \
                mask.reshape(-1, 1).to(deltas.dtype)
            deltas = torch.cat([deltas, m], dim=1)
        elif mask is not None:
            deltas = deltas * mask.reshape(-1, 1).to(deltas.dtype)
        wire = deltas if deltas.dtype == self.wire_dtype else deltas.to(self.wire_dtype)
        opt = op or self.table.optimizer
        can_defer = (not plan.fixed and plan.valid is None and not return_updated and opt != "fn"
                     and self.table.device.type == "cuda")
        into = self._defer_into
        if (defer or into is not None) and can_defer and self.owner_stream is None:
            with stage("ps.push-a2a", self.timer):
                recv, work = self.comm.all_to_all_async(wire.contiguous(), plan.send_splits, plan.recv_splits)
            pp = PendingPush(plan, recv, work, opt, lr)
            if into is not None and not defer:
                into.append((self, pp))
                return None
            return pp
        if self.owner_stream is not None and can_defer:
            # owner-stream mode: the push travels while the compute stream goes on; the
            # owner stream waits for it and applies (after every earlier serve / apply)
            self._compute_stream = torch.cuda.current_stream(self.table.device)
            with stage("ps.push-a2a", self.timer):
                recv, work = self.comm.all_to_all_async(wire.contiguous(), plan.send_splits, plan.recv_splits)
            with torch.cuda.stream(self.owner_stream):
                if plan.key_work is not None:  # a push without a pull: its keys' transfer
                    plan.key_work.wait()
                    plan.key_work = None
                self._owner_enter(work, recv, plan.recv_keys)
                self._apply_pushed(plan, recv, opt, lr, mark=plan.recv_rows is None)
            return None
        with stage("ps.push-a2a", self.timer):
            recv = self.comm.all_to_all(wire.contiguous(), plan.send_splits, plan.recv_splits)
        self.owner_sync()  # an apply on the compute stream: after every owner-stream serve / apply
        if plan.key_work is not None:
            plan.key_work.wait()
            plan.key_work = None
        recv_keys = self._apply_pushed(plan, recv, op or self.table.optimizer, lr, mark=plan.recv_rows is None)
        if return_updated:
            if not sum(plan.recv_splits):  # nothing arrived at this shard (host-known sizes)
                return None
            if self.masked_push or plan.fixed:  # skipped / padding rows drop out when the consumer reads
                k = recv_keys.long().clamp_min(0)
                return MaskedPair(self.table.global_ids(k), self.table.weight[k], recv_keys >= 0)
            return self.table.global_ids(recv_keys), self.table.weight[recv_keys.long()]
        return None

    def apply_pending(self, pp: "PendingPush") -> None:
        """Wait (on the current stream) for a deferred push's transfer and apply it."""
        if pp.work is not None:
            pp.work.wait()
        if pp.plan.key_work is not None:
            pp.plan.key_work.wait()
            pp.plan.key_work = None
        self._apply_pushed(pp.plan, pp.recv, pp.opt, pp.lr, mark=pp.plan.recv_rows is None)

    def _apply_pushed(self, plan: PullPlan, recv: torch.Tensor, opt: str, lr: float, mark: bool) -> torch.Tensor:
        """Apply one push's received rows (stage 9); returns the local rows written (-1:
        skipped)."""
        D = self.table.dim
        fresh = None
        # served by this plan: the rows exist and were marked touched when served (mark)
        if plan.recv_rows is not None:
            rows = plan.recv_rows
        else:  # a push without a pull (push_keys, model load)
            rows, fresh = self.table.rows_for(plan.recv_keys, push=True)
        recv_keys = rows
        if plan.valid is not None:  # static plan: the padding rows are never applied
            if plan.push_rows is not None and rows is plan.recv_keys:  # dense: built with the plan
                recv_keys = plan.push_rows
            else:
                recv_keys = torch.where(plan.valid, recv_keys, torch.full_like(recv_keys, -1))
        if self.masked_push:
            valid = recv[:, D] > 0.5
            recv = recv[:, :D].contiguous()
            recv_keys = torch.where(valid, recv_keys, torch.full_like(recv_keys, -1))
        if plan.valid is not None:
            self._count_lazy("pushes", plan.valid, total=plan.n_valid)
        elif plan.fixed:
            self._count_lazy("pushes", recv_keys >= 0)
        else:
            self._stats["pushes"] += plan.n_unique
        with stage("ps.apply", self.timer):
            # (a request plan repeats keys inside a segment: atomic add)
            seg_add = opt == "add" and len(plan.recv_splits) <= 16 and plan.unique and plan.recv_unique
            if opt == "fn":  # user rule: sequential over the source segments (keys repeat across them)
                if fresh is not None:  # the id is absent only for its first push, in segment order
                    fresh = self._first_fresh(recv_keys, fresh)
                off = 0
                for n in plan.recv_splits:
                    if n:
                        self.table.apply_rows(recv_keys[off:off + n], recv[off:off + n], lr=lr, op=opt,
                                              fresh=None if fresh is None else fresh[off:off + n])
                    off += n
            elif seg_add or opt in ("adagrad", "set", "add_renorm"):
                # Keys are unique within each source's segment but may repeat across
                # sources; non-atomic rules (adagrad's accumulator RMW, set, renorm)
                # therefore apply segment by segment.  ``add`` does the same with a
                # plain read-modify-write (add_unique) instead of one float atomic per
                # element (the atomic apply ran at ~1 TB/s: 480 us for 2M dim-64
                # rows, profiles/r1_capacity_kernel_stats.csv; narrow rows are worse).
                off = 0
                for n in plan.recv_splits:
                    if n:
                        self.table.apply_rows(recv_keys[off:off + n], recv[off:off + n], lr=lr,
                                              op="add_unique" if seg_add else opt, mark=mark)
                    off += n
            else:
                self.table.apply_rows(recv_keys, recv, lr=lr, op=opt, mark=mark)
        return recv_keys

    @staticmethod
    def _first_fresh(rows: torch.Tensor, fresh: torch.Tensor) -> torch.Tensor:
        """Per request: is it the FIRST request (lowest index) of a row any of
        whose requests found the id absent?  Sort-based, no host sync."""
        n = rows.numel()
        if n == 0:
            return fresh.bool()
        order = torch.argsort(rows.long(), stable=True)
        sr = rows.long()[order]
        first = torch.ones(n, dtype=torch.bool, device=rows.device)
        first[1:] = sr[1:] != sr[:-1]
        grp = torch.cumsum(first.long(), 0) - 1
        gf = torch.zeros(n, dtype=torch.long, device=rows.device)
        gf.scatter_reduce_(0, grp, fresh.long()[order], reduce="amax")
        out = torch.empty(n, dtype=torch.bool, device=rows.device)
        out[order] = first & (gf[grp] > 0) & (sr >= 0)
        return out

    def note_local_push(self, plan: PullPlan) -> None:
        """Book a push the worker applied to this (local, additive) shard itself
        (world 1: its compute kernel added the deltas to ``recv_keys``' rows)."""
        if self.comm.world != 1 or getattr(self.table, "optimizer", "") != "add":
            raise ValueError("local pushes need world 1 and an additive table")
        if plan.valid is not None:  # static plan: its padding rows are never pushed
            self._count_lazy("pushes", plan.valid, total=plan.n_valid)
        else:
            self._stats["pushes"] += plan.n_unique

    def reduce_requests(self, plan: PullPlan, deltas: torch.Tensor, op: str = "add",
                        mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Per-request ``[B, D]`` deltas -> per-unique-key ``[U, D]``: summed for
        additive rules, the LAST request's value for ``set`` (last writer wins,
        the order a per-record PS would apply them in).  ``mask[b] = False``
        drops request ``b``."""
        D = deltas.shape[1] if deltas.dim() > 1 else 1
        d2 = deltas.reshape(deltas.shape[0], D).float()
        pos = plan.pos.long()
        if op == "set":
            rid = torch.arange(pos.numel(), device=pos.device)
            if mask is not None:
                rid = torch.where(mask, rid, torch.full_like(rid, -1))
            last = torch.full((plan.n_unique,), -1, dtype=torch.int64, device=pos.device)
            last.scatter_reduce_(0, pos, rid, reduce="amax")
            if mask is not None and bool((last < 0).any()):
                raise ValueError("set-push with a masked key: every unique key needs a value")
            return d2[last.clamp_min(0)].contiguous()
        out = torch.zeros((plan.n_unique, D), dtype=torch.float32, device=d2.device)
        if mask is not None:
            d2 = d2 * mask.view(-1, 1).to(d2.dtype)
        out.index_add_(0, pos, d2)
        return out

    def push_keys(self, keys: torch.Tensor, deltas: torch.Tensor, lr: float = 0.0, op: Optional[str] = None,
                  return_updated: bool = False):
        """Push to arbitrary keys (not a pulled plan): plans them (host waits on
        the counts), pre-reduces duplicates and applies (always a de-duplicating plan:
        ``set`` needs one value per key)."""
        plan = self.plan(keys, dedup=True)
        opt = op or self.table.optimizer
        red = self.reduce_requests(plan, deltas, "set" if opt == "set" else "add")
        return self.push(plan, red, lr=lr, op=opt, return_updated=return_updated)

    def load(self, ids: torch.Tensor, values: torch.Tensor) -> None:
        """Model load (``transformWithModelLoad``, ``M/FlinkParameterServer.scala:377-566``):
        every rank passes the ``(id, value)`` records IT received; they are routed
        to their owning shards and written there (last record of an id wins).
        Collective."""
        vals = values.to(device=self.table.device, dtype=torch.float32).reshape(ids.numel(), self.table.dim)
        self.push_keys(ids, vals, op="set")

    def pull_values(self, keys: torch.Tensor) -> torch.Tensor:
        """Convenience: fp32 ``[B, D]`` values for every request (expanded)."""
        rows, plan = self.pull(keys)
        return rows.float()[plan.pos.long()]
