"""Online MF-SGD on the tensor engine (the north-star workload).

Same model and data flow as ``psOnlineMF``
(``M/matrix/factorization/PSOnlineMatrixFactorization.scala:39-75``):

* ratings are partitioned by ``user % W`` (``:62-64``), so each worker owns
  the user vectors of its users (worker-resident table, P3);
* item vectors live on the PS, hash-sharded ``item % W``, updated by pushing
  deltas that the PS adds (``SimplePSLogic`` with vector sum, ``:58-60``);
* per rating: ``e = r - u.i``, ``u += lr*e*i``, push ``lr*e*u`` to the item
  (``SGDUpdater``), init U[-0.01, 0.01) (``RangedRandomFactorInitializer``).

Execution per micro-batch of B ratings on each GPU:

* ``W == 1`` — the item shard is local: one fused kernel reads u and i,
  stores u (Hogwild inside the batch; optional atomics) and atomically adds
  di into the item row (``ops.mf_sgd_local``).  No wire buffers at all.
* ``W > 1``, ``exchange="rotate"`` (default) — the item shards travel between
  the GPUs instead of rows travelling to the ratings
  (``parallel.rotation.RingRotation``, stratified SGD): the micro-batch is
  partitioned by item block on the GPU, then 2W sub-steps each run the SGD on
  the resident blocks while the next ones arrive from the neighbours -- two
  counter-rotating rings of quarter-shard blocks by default (``rotation="bidir"``:
  both directions of two xGMI links), or one ring (``"ring"``).  No dedup, no
  pulls, no staleness.  ``emulate_world=N`` runs rank 0's schedule of an N-GPU
  job on one GPU with every block resident (the per-GPU compute at N).
* ``W > 1``, ``exchange="ps"`` — ``TensorPS.pull`` (dedup + 2 all-to-alls),
  fused SGD on the pulled rows accumulating per-unique-item deltas
  (``ops.mf_sgd_pulled``), ``TensorPS.push`` (all-to-all + apply); the pull of
  batch k+1 overlaps the SGD of batch k.  The reference's protocol, for
  workloads whose model does not fit the rotation (and the parity tests).

Throughput unit: rating-SGD updates/s (each updates one user row and one item
row of ``dim`` floats), see BASELINE.md.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import os

import torch
import torch.distributed

from ... import ops
from ...parallel.comm import Comm
from ...parallel.rotation import EmulatedRotation, RingRotation, layout_world, shard_halves
from ...parallel.rotation import block_rows as block_rows_of
from ...api.batched import BatchedWorkerLogic
from ...parallel.table import ShardedTable
from ...parallel.tensor_ps import TensorPS
from ...utils.metrics import Counters
from ...utils.tracing import stage


@dataclass
class MFConfig:
    num_users: int = 10_000_000
    num_items: int = 1_000_000
    dim: int = 64
    learning_rate: float = 0.01
    lam: float = 0.0
    range_min: float = -0.01
    range_max: float = 0.01
    seed: int = 0
    user_update: str = "auto"         # "store" (Hogwild, plain accesses) | "sc1" (Hogwild, write-through user
                                      # rows: ~half the lost user updates, profiles/r4_hogwild.md) | "atomic"
                                      # (exact: no lost update -- the tiled kernel adds every user delta with
                                      # float atomics; the flat kernel where the tiled one does not apply) |
                                      # "auto" = "store" at EVERY world size: one semantics for the whole
                                      # 1 -> N curve (bench.py reports the lost fraction and the exact
                                      # rate beside it; profiles/r6_exact_user_rows.md)
    wire_dtype: str = "fp32"          # "fp32" | "bf16" (pull answers + pushed deltas)
    force_ps_path: bool = False       # run the pull/push protocol even when the shard is local
    sgd_mode: str = "auto"            # "auto" | "tiled" | "flat" | "grouped"
    pipeline: bool = True             # overlap pull(k+1) all-to-all with SGD(k) (remote PS path)
    fuse_local_push: bool = True      # PS path, world 1, identity plan: the tiled SGD updates the served
                                      # shard rows in place -- the push applied by the kernel (no delta
                                      # buffer, second row read or apply pass); False: delta mode + apply
    prefetch_partition: bool = True   # tiled: bucket batch k+1 on a side stream during the SGD of k
    negative_sample_rate: int = 0     # implicit feedback: negatives (rating 0) per rating
    user_memory: int = 128            # per-user ring of recent items excluded from the negatives
    user_phases: int = 0              # tiled: run the SGD in P user-range phases (0 = auto: ~2.5M users
                                      # per phase, so a launch's user rows mostly hit the Infinity Cache)
    graph_capture: bool = False       # tiled, W = 1: replay each batch size's step as one hipGraph
                                      # (launch-bound small batches; disables the prefetch)
    exchange: str = "auto"            # W > 1: "rotate" (item-block ring, default) | "ps" (pull/push);
                                      # W = 1: "local" (default); "rotate"/"ps" run those paths without peers
    rotation: str = "bidir"           # rotate: "bidir" (two counter-rotating rings) | "ring" (one ring)
    overlap_substeps: object = "auto"  # rotate, tiled: sub-steps alternate two compute streams, so sub-step
                                      # s + 1 (other item blocks) fills the tail of s (same users: Hogwild).
                                      # "auto": from 4 ranks on -- with 2 ranks a block takes ~40 % of a
                                      # sub-step on the link and the overlap eats that slack
                                      # (profiles/r4_emulate_overlap.jsonl)
    emulate_world: int = 0            # W = 1, rotate: rank 0's share of an N-rank job (users / schedule)
    emulate_link_gbps: float = 0.0    # emulate_world: model the transfers on links of this rate (0: none)
    emulate_latency_us: float = 5.0   # emulate_world: per-message link latency


    def user_seed(self) -> int:
        """Hash-init seed of the user table (the per-record apps' ``init="hash"``
        user side: seed ^ USER_SEED_XOR), so both engines start from one model."""
        from .core import USER_SEED_XOR

        return (self.seed ^ USER_SEED_XOR) & 0xFFFFFFFF

    def item_seed(self) -> int:
        return self.seed & 0xFFFFFFFF


_WIRE = {"fp32": torch.float32, "bf16": torch.bfloat16}

#: user rows per SGD phase (auto ``user_phases``): 2.5M x 64 fp32 = 640 MB
PHASE_USERS = 2_500_000


class DistributedMF:
    def __init__(self, cfg: MFConfig, comm: Optional[Comm] = None):
        self.cfg = cfg
        self.comm = comm or Comm()
        W, r, dev = self.comm.world, self.comm.rank, self.comm.device
        init = ("uniform", cfg.range_min, cfg.range_max)
        self.emulated = cfg.emulate_world > 1
        if self.emulated and (W != 1 or cfg.exchange not in ("rotate", "auto")):
            raise ValueError("emulate_world runs the rotation schedule of N ranks in ONE process")
        Wn = cfg.emulate_world if self.emulated else W  # the job's world (emulated or real)
        # worker-resident user shard: users u with u % W == r, local row u // W
        self.users = ShardedTable(cfg.num_users, cfg.dim, r, Wn, "hash", init, cfg.user_seed(), dev,
                                  track_touched=False)
        # PS item shard
        self.items = ShardedTable(cfg.num_items, cfg.dim, r, W, "hash", init, cfg.item_seed(), dev, optimizer="add")
        self.ps = TensorPS(self.items, self.comm, _WIRE[cfg.wire_dtype])
        uu = cfg.user_update
        if uu == "auto":
            # the same user-row semantics at every world size (round 5 switched to the exact
            # mode at N > 1, so a scaling curve measured a mode change).  The reference updates
            # a user's vector sequentially inside its one worker
            # (M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:41-55):
            # "atomic" loses no user update and costs ~2x the step on MI355X (float atomics are
            # executed memory-side at ~1.3 TB/s whatever the working set,
            # profiles/r6_exact_user_rows.md); bench.py times both modes on every line
            uu = "store"
        if uu not in ("store", "sc1", "atomic"):
            raise ValueError(f"user_update must be 'auto', 'store', 'sc1' or 'atomic', not {cfg.user_update!r}")
        #: the resolved user-row update mode
        self.user_update = uu
        self.user_atomic = uu == "atomic"
        self.user_sc1 = uu == "sc1" and dev.type == "cuda"
        #: tiled kernel's user-row mode (ops.USER_MODES): plain / write-through / atomic deltas
        self.user_mode = ops.USER_MODES[uu] if dev.type == "cuda" or uu == "atomic" else 0
        exchange = cfg.exchange
        if exchange == "auto":
            exchange = "ps" if cfg.force_ps_path else ("rotate" if Wn > 1 else "local")
        if exchange not in ("rotate", "ps", "local") or (exchange == "local" and W > 1):
            raise ValueError(f"exchange {cfg.exchange!r} invalid at world size {W}")
        self.exchange = exchange
        # SGD kernel:
        #  "tiled"   item rows staged in LDS per tile of R rows, ratings bucketed
        #            by tile, item deltas by LDS atomics -- no global item atomics
        #            (mf_tiled.hip; default where the dim/table size fit);
        #  "flat"    one rating per lane group, item deltas by 256-B global float
        #            atomics (atomic-rate bound: 3.9e9 ratings/s, profiles/README.md);
        #  "grouped" ratings sorted by item, each item row updated in registers
        #            (exact per-item order; latency bound, 2.8e9/s).
        # local: the table as 2 blocks (halves) of one shard; rotate: 2W blocks; ps:
        # the pulled rows of a micro-batch (<= num_items unique items) as one block
        tile_w = layout_world(Wn, cfg.rotation) if exchange == "rotate" else 1
        block_rows = cfg.num_items if exchange == "ps" else max(block_rows_of(cfg.num_items, tile_w))
        tile_R = ops.tile_rows_for(cfg.dim, block_rows, tile_w)
        mode = cfg.sgd_mode
        # exact user rows in the tiled kernel: 8-B records (< 2^24 users per shard) and a
        # user table < 4 GiB (32-bit offsets); otherwise the flat atomic kernel
        users_local = -(-cfg.num_users // Wn)
        tiled_atomic_ok = users_local < (1 << 24) and users_local * cfg.dim * 4 < 0xFFFFFFFF
        if mode == "auto":
            mode = "tiled" if (tile_R is not None and (not self.user_atomic or tiled_atomic_ok)) else "flat"
        if mode == "tiled" and (tile_R is None or (self.user_atomic and not tiled_atomic_ok)):
            raise ValueError("sgd_mode 'tiled' needs dim in ops.TILED_DIMS, a table small enough for the LDS "
                             "bucket counters and (user_update='atomic') < 2^24 users and < 4 GiB per shard")
        if mode == "grouped" and exchange == "rotate":
            raise ValueError("sgd_mode 'grouped' is not available with the rotation exchange")
        self.sgd_mode = mode
        self.grouper = ops.CSRGrouper(dev)
        if mode == "tiled":
            self.tile_R = tile_R
            self.tile_T = -(-block_rows // tile_R)
            # two partition buffers: with prefetch the partition of batch k+1 runs on a
            # side stream while batch k's SGD runs (one micro-batch of latency, flush()
            # completes it; same SGD order)
            rec8 = self.users.n_local < (1 << 24)  # 8-B rating records (user index in 24 bits)
            if self.user_sc1 and not (rec8 and self.U.numel() * 4 < 0xFFFFFFFF):
                raise ValueError("user_update='sc1' addresses the user shard with 32-bit byte offsets: "
                                 "< 2^24 users and < 4 GiB per shard")
            # user phases: ratings also bucketed by local user range, each phase's
            # launches touch ~2.5M user rows (640 MB) instead of all of them --
            # measured 1.67 ms x 4 vs 7.34 ms of SGD per 64M ratings at 10M users
            # (profiles/r1_mf_user_phases.md)
            P = cfg.user_phases or -(-self.users.n_local // PHASE_USERS)
            while P > 1 and P * 2 * tile_w * self.tile_T > ops.TILE_MAX_BUCKETS:
                P -= 1
            self.user_phases = max(1, P)
            upp = -(-self.users.n_local // self.user_phases)
            halves = [cfg.num_items] if exchange == "ps" else shard_halves(cfg.num_items, tile_w)
            # ps: a batch covering the key space gets an identity plan (pulled row = item id,
            # ``TensorPS.identity_for``), so its partition can be staged when the batch is
            # RECEIVED, beside the SGD of an earlier batch: with the pipeline (staleness 1)
            # two received batches wait for their compute -> three partition buffers
            ps_spec = exchange == "ps" and cfg.prefetch_partition and dev.type == "cuda"
            n_tilers = 2 if exchange != "ps" else (3 if ps_spec else 1)
            bounds = dict(num_users=self.users.n_local, num_items=cfg.num_items)
            self._tilers = [ops.TilePartitioner(tile_w, halves, tile_R, self.tile_T, dev, rec8=rec8,
                                                phases=self.user_phases, users_per_phase=upp, **bounds)
                            for _ in range(n_tilers)]
            # PS path, identity plans: the partition's count pass marks the items a batch
            # rates (one flag array per partition buffer) -- the plan's presence flags, so
            # the PS needs no marking pass over the 64M keys of its own
            self._presence = [torch.zeros(cfg.num_items, dtype=torch.uint8, device=dev) for _ in range(n_tilers)] \
                if ps_spec else None
            self._tiler_i = 0
            self._graphs = {} if (cfg.graph_capture and dev.type == "cuda" and exchange == "local") else None
            self._prefetch = (cfg.prefetch_partition and dev.type == "cuda" and self._graphs is None
                              and exchange != "ps")
            self._ps_spec = ps_spec
            # the PS path's own partition (batches without an identity plan)
            self._ps_tiler = self._tilers[0] if not ps_spec else \
                ops.TilePartitioner(tile_w, halves, tile_R, self.tile_T, dev, rec8=rec8, phases=self.user_phases,
                                    users_per_phase=upp, **bounds)
            # the partition of batch k+1 runs on a side stream beside the SGD of batch k
            # (a priority stream for the SGD and CU-masked streams splitting the CUs
            # between them were measured slower and removed, profiles/r2_partition.md)
            # FPS_PART_PRIORITY (A/B knob): the partition's side-stream priority (-1: high)
            prio = int(os.environ.get("FPS_PART_PRIORITY", "0"))
            self._side = torch.cuda.Stream(dev, priority=prio) if (self._prefetch or ps_spec) else None
            # rotation sub-steps on alternating streams (``MFConfig.overlap_substeps``)
            ov = cfg.overlap_substeps
            if ov == "auto":
                ov = Wn >= 4
            elif not isinstance(ov, bool):
                raise ValueError(f"overlap_substeps must be True, False or 'auto', not {ov!r}")
            self._overlap = ov and self.exchange == "rotate" and dev.type == "cuda"
            self._aux = torch.cuda.Stream(dev) if self._overlap else None
            self._staged = None
            h0 = shard_halves(cfg.num_items, 1)[0]
            self._local_blocks = [self.items.weight[:h0], self.items.weight[h0:]]
        if self.exchange == "rotate":
            if self.emulated:
                self.rot = EmulatedRotation(self.items.weight, cfg.num_items, Wn, cfg.rotation,
                                            link_gbps=cfg.emulate_link_gbps or None,
                                            latency_us=cfg.emulate_latency_us)
            else:
                self.rot = RingRotation(self.comm, self.items.weight, cfg.num_items, cfg.rotation)
            self.rot_w = tile_w  # hash shards of the block layout the ratings are bucketed by
            self.partitioner = ops.RotationPartitioner(tile_w, torch.tensor(shard_halves(cfg.num_items, tile_w)),
                                                       dev)
            # rows are updated in rotating buffers: remember which items were rated
            # so the close-time dump still covers exactly the touched parameters
            self._seen = torch.zeros(cfg.num_items, dtype=torch.uint8, device=dev)
        self.pipeline = cfg.pipeline and self.exchange == "ps"
        if self.exchange == "ps":
            # the reference's pull / push protocol through the public batched API on
            # the tensor engine: a worker over this model's user rows + the item
            # shard as a SimplePSLogic(add) device logic.  pipeline = staleness 1: the
            # pull of batch k+1 (counts exchanged one call earlier, its row
            # all-to-all in flight) overlaps the SGD of batch k.
            from ...core.tensor_engine import TensorRuntime
            from ...ps.device_logics import DeviceSimplePSLogicWithClose

            logic = DeviceSimplePSLogicWithClose(cfg.num_items, cfg.dim, table=self.items, ps=self.ps)
            if self.sgd_mode == "tiled" and self._ps_spec:
                # the delta-mode SGD only reads the pulled rows, and the staged partition
                # (not the plan's positions) addresses them: the world-1 identity plan may
                # serve the shard itself and keep the batch's key tensor as is
                self.ps.zero_copy_identity = True
                self.ps.keys_stable = True
            self.runtime = TensorRuntime(self.comm, staleness=1 if self.pipeline else 0)
            self.runtime.start(_MFPSWorker(self), logic)
        if cfg.negative_sample_rate > 0:
            # PSOnlineMatrixFactorizationWorker.scala:70-79: per rating, negativeSampleRate
            # items (rating 0) drawn among the items this worker has seen, not among the
            # user's last userMemory items.  Device state: per-user ring + cursor, the
            # worker's known-item list; the negatives join the batch as extra ratings.
            n_u = self.users.n_local
            self._ring = torch.full((n_u * cfg.user_memory,), -1, dtype=torch.int32, device=dev)
            self._ring_cursor = torch.zeros(n_u, dtype=torch.int32, device=dev)
            self._known_flag = torch.zeros(cfg.num_items, dtype=torch.int32, device=dev)
            self._known = torch.zeros(cfg.num_items, dtype=torch.int32, device=dev)
            self._known_count = torch.zeros(1, dtype=torch.int32, device=dev)
            self._neg_counter = 0
        self._part_delay_us = float(os.environ.get("FPS_PART_DELAY_US", "0"))
        self.updates = 0
        #: observability: ``timer`` (a ``utils.metrics.StageTimer``, set by
        #: bench.py --metrics-jsonl) times every stage with HIP events; the counters
        #: are host-side tallies of what was enqueued (no device sync)
        self.timer = None
        self.counters = Counters()

    @property
    def U(self):
        return self.users.weight

    @property
    def I(self):
        return self.items.weight

    def set_user_update(self, mode: str) -> None:
        """Switch the tiled kernel's user-row mode between steps ("store" / "sc1" /
        "atomic"): the same model, partition and schedule, only the user-row write differs
        (bench.py times the exact mode beside the Hogwild one).  Call after ``flush()``."""
        if self.sgd_mode != "tiled":
            raise ValueError("set_user_update switches the tiled kernel's user-row mode")
        if mode not in ("store", "sc1", "atomic"):
            raise ValueError(f"user_update must be 'store', 'sc1' or 'atomic', not {mode!r}")
        dev = self.comm.device
        if mode in ("sc1", "atomic") and dev.type == "cuda" and not (
                self.users.n_local < (1 << 24) and self.U.numel() * 4 < 0xFFFFFFFF):
            raise ValueError(f"user_update={mode!r} needs < 2^24 users and < 4 GiB per shard")
        self.user_update = mode
        self.user_atomic = mode == "atomic"
        self.user_sc1 = mode == "sc1" and dev.type == "cuda"
        self.user_mode = ops.USER_MODES[mode] if dev.type == "cuda" or mode == "atomic" else 0

    def step(self, uid_local: torch.Tensor, iid: torch.Tensor, rating: torch.Tensor):
        """One micro-batch. ``uid_local`` = row in this worker's user shard,
        ``iid`` = global item id (int32), ``rating`` fp32."""
        c = self.cfg
        grouped = self.sgd_mode == "grouped"
        uid_local, iid, rating = uid_local.contiguous(), iid.contiguous(), rating.contiguous()
        if ops.DEBUG:  # FPS_DEBUG=1: range checks before any kernel sees the batch
            ops.check_index(uid_local, self.users.n_local, "MF step uid_local")
            ops.check_index(iid, c.num_items, "MF step iid")
        if c.negative_sample_rate > 0:
            uid_local, iid, rating = self._with_negatives(uid_local, iid, rating)
        tiled = self.sgd_mode == "tiled" and self.exchange != "ps"  # ps: tiled inside _compute_push
        if tiled and self._graphs is not None:
            self._graph_step(uid_local, iid, rating)
        elif tiled:
            # bucket this batch (side stream when prefetching) and run the SGD of
            # the batch staged by the previous call: the partition of k+1 overlaps
            # the SGD of k; the order of the SGD steps is unchanged
            staged = self._stage_partition(uid_local, iid, rating)
            if self._prefetch:
                prev, self._staged = self._staged, staged
                if prev is not None:
                    self._tiled_sgd(prev)
            else:
                self._tiled_sgd(staged)
        elif self.exchange == "local":
            with stage("mf.sgd", self.timer):
                if grouped:
                    ptr, order = self.grouper.run(iid, self.items.n_local)
                    ops.mf_sgd_grouped(self.U, self.I, uid_local, rating, ptr, order, c.learning_rate, c.lam)
                else:
                    ops.mf_sgd_local(self.U, self.I, uid_local, iid, rating, c.learning_rate, c.lam,
                                     self.user_atomic)
        elif self.exchange == "rotate":
            seen = self._seen if self.items.touched is not None else None
            with stage("mf.partition", self.timer):
                ptr, u, row, r = self.partitioner.run(uid_local, iid, rating, seen)
            n = uid_local.numel()
            for _ in range(self.rot.K):
                with stage("mf.rotate.begin", self.timer):
                    self.rot.begin()  # transfer of the next blocks overlaps this sub-step
                with stage("mf.sgd", self.timer):
                    for g, blk in self.rot.active_blocks():
                        ops.mf_sgd_local_seg(self.U, blk, u, row, r, ptr, g, n, c.learning_rate, c.lam,
                                             self.user_atomic)
                with stage("mf.rotate.end", self.timer):
                    self.rot.end()
        else:  # PS path: one micro-batch through the tensor engine
            self.runtime.submit((uid_local, iid, rating))
        self.updates += uid_local.numel()
        self.counters.add("ratings", uid_local.numel())
        self.counters.add("micro_batches")
        if ops.DEBUG:  # FactorIsNotANumberException, M/matrix/factorization/utils/Vector.scala:78-80
            from .core import FactorIsNotANumberException

            ops.check_finite(self.U, "user factors", FactorIsNotANumberException)
            if self.exchange != "rotate":
                ops.check_finite(self.I, "item factors", FactorIsNotANumberException)

    def _with_negatives(self, uid, iid, rating):
        """Append ``negative_sample_rate`` implicit negatives (rating 0) per rating."""
        c = self.cfg
        k = c.negative_sample_rate
        ops.ring_push(self._ring, self._ring_cursor, uid, iid, c.user_memory)
        ops.known_append(self._known_flag, self._known, self._known_count, iid)
        negs = ops.sample_uniform_reject(uid.numel(), k, c.num_items, iid, uid, self._ring, c.user_memory,
                                         seed=c.seed + 7 * self.comm.rank, counter=self._neg_counter,
                                         device=uid.device, known=self._known, known_count=self._known_count)
        self._neg_counter += 1
        return (torch.cat([uid, uid.repeat_interleave(k)]), torch.cat([iid, negs]),
                torch.cat([rating, torch.zeros(uid.numel() * k, dtype=rating.dtype, device=rating.device)]))

    def _graph_step(self, uid_local, iid, rating):
        """One local tiled step as a captured hipGraph (partition + SGD kernels,
        no host sync inside), one graph per batch size.  The first batch of a
        size runs eagerly (warm-up: buffers allocated) and is captured after."""
        n = uid_local.numel()
        entry = self._graphs.get(n)
        if entry is not None:
            graph, static = entry
            for dst, src in zip(static, (uid_local, iid, rating)):
                dst.copy_(src)
            graph.replay()
            return
        dev = self.U.device
        static = [uid_local.clone(), iid.clone(), rating.clone()]
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # eager warm-up = this batch's real step
            self._tiled_sgd(self._stage_partition(*static))
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):  # capture only: nothing executes here
            self._tiled_sgd(self._stage_partition(*static))
        self._graphs[n] = (graph, static)

    def _stage_partition(self, uid_local, iid, rating):
        """Tile partition of one batch into the next of the two partition buffers;
        returns ``(ptr, rec, ready_event)`` (PS path, identity plans: the count pass also
        marks the batch's items in this buffer's presence flags, ``self._presence[i]``)."""
        seen = self._seen if (self.exchange == "rotate" and self.items.touched is not None) else None
        i = self._tiler_i
        tiler = self._tilers[i]
        self._tiler_i = (self._tiler_i + 1) % len(self._tilers)
        if self._presence is not None:
            seen = self._presence[i]
        if self._side is None:
            with stage("mf.partition", self.timer):
                ptr, rec = tiler.run(uid_local, iid, rating, seen)
            return ptr, rec, None
        main = torch.cuda.current_stream(self.U.device)
        self._side.wait_stream(main)  # inputs written, and this buffer's previous SGD done
        with torch.cuda.stream(self._side):
            if self._part_delay_us > 0:
                # A/B knob (FPS_PART_DELAY_US): let the SGD launch that starts with this
                # partition fill the CUs first
                from ...parallel.vworld import _Sleep

                _Sleep.us(self.U.device, self._part_delay_us)
            if self._presence is not None:
                seen.zero_()
            with stage("mf.partition", self.timer):  # timed on the side stream
                ptr, rec = tiler.run(uid_local, iid, rating, seen)
            ev = torch.cuda.Event()
            ev.record(self._side)
        for t in (uid_local, iid, rating):
            t.record_stream(self._side)
        return ptr, rec, ev

    def _tiled_sgd(self, staged):
        c = self.cfg
        ptr, rec, ev = staged
        if ev is not None:
            torch.cuda.current_stream(self.U.device).wait_event(ev)
        if self.exchange == "local":
            b0, b1 = self._local_blocks
            with stage("mf.sgd", self.timer):
                for p in range(self.user_phases):  # both item blocks of a phase in one launch
                    ops.mf_sgd_tiled_pair(self.U, b0, b1, rec, ptr, 2 * p, self.tile_T, self.tile_R,
                                          c.learning_rate, c.lam, user_mode=self.user_mode)
            return
        nb = 2 * self.rot_w  # item blocks per user phase in the partition layout

        def sub_step():
            act = self.rot.active_blocks()
            for p in range(self.user_phases):
                if len(act) == 2:  # one block of each ring: disjoint items, one launch
                    (g0, b0), (g1, b1) = act
                    ops.mf_sgd_tiled_pair(self.U, b0, b1, rec, ptr, p * nb + g0, self.tile_T, self.tile_R,
                                          c.learning_rate, c.lam, block1=p * nb + g1, user_mode=self.user_mode)
                else:
                    (g0, b0), = act
                    ops.mf_sgd_tiled(self.U, b0, rec, ptr, p * nb + g0, self.tile_T, self.tile_R,
                                     c.learning_rate, c.lam, user_mode=self.user_mode)

        if not self._overlap:
            for _ in range(self.rot.K):
                with stage("mf.rotate.begin", self.timer):
                    self.rot.begin()  # transfer of the next blocks overlaps this sub-step
                with stage("mf.sgd", self.timer):
                    sub_step()
                with stage("mf.rotate.end", self.timer):
                    self.rot.end()
            return
        # Sub-steps alternate two compute streams: sub-step s + 1 updates other item
        # blocks, so it may start in the tail of s (a launch of ~2k workgroups leaves the
        # CUs half idle for its last round).  Stream roles per sub-step s on `cur`:
        #   begin(s) is posted from the stream of s - 1: its sends carry the blocks s - 1
        #     finished, so they must follow s - 1 and only s - 1;
        #   end(s) waits for the transfers from the stream of s + 1, the one that reads
        #     the arriving blocks.
        # The first sub-step's blocks leave their rest state on `main`; `main` joins the
        # other stream after the last sub-step.
        main = torch.cuda.current_stream(self.U.device)
        aux = self._aux
        aux.wait_stream(main)  # the partition (staged event) and the previous step
        streams = (main, aux)
        for s in range(self.rot.K):
            cur, prev, nxt = streams[s % 2], streams[(s - 1) % 2], streams[(s + 1) % 2]
            with torch.cuda.stream(cur if s == 0 else prev):
                with stage("mf.rotate.begin", self.timer):
                    self.rot.begin()
            if s == 0:
                aux.wait_stream(main)  # sub-step 1 on aux reads blocks that left rest on main
            with torch.cuda.stream(cur):
                with stage("mf.sgd", self.timer):
                    sub_step()
            with torch.cuda.stream(nxt):
                with stage("mf.rotate.end", self.timer):
                    # the next sub-step's stream waits for the arriving blocks; this one
                    # too: it posts the next transfers, whose receives reuse the buffers
                    # these transfers' sends read
                    self.rot.end(also=(cur,))
        main.wait_stream(aux)

    def _item_deltas(self, rows, pos, n_unique, uid_local, rating, staged=None):
        """SGD of one micro-batch on its pulled item rows ``rows[pos[b]]``; returns
        the per-unique-item deltas to push (user rows are updated in place).
        ``staged``: the batch's partition by item id, staged when it was received
        (valid when the plan is the identity: pulled row = item id)."""
        c = self.cfg
        if self.sgd_mode == "tiled":
            # tile-grouped SGD on the pulled rows (one block, no item atomics) in the
            # kernel's delta mode: the rows stay as pulled and the kernel writes what
            # the micro-batch added to each row -- the pushed delta -- directly
            rows = rows if rows.dtype == torch.float32 else rows.float()
            delta = torch.empty_like(rows)  # every row written by the first phase's launch
            if staged is not None:
                ptr, rec, ev = staged
                if ev is not None:
                    torch.cuda.current_stream(self.U.device).wait_event(ev)
            else:
                ptr, rec = self._ps_tiler.run(uid_local, pos, rating)
            with stage("mf.sgd", self.timer):
                for p in range(self.user_phases):
                    ops.mf_sgd_tiled(self.U, rows, rec, ptr, 2 * p, self.tile_T, self.tile_R, c.learning_rate,
                                     c.lam, delta=delta, delta_init=p == 0, user_mode=self.user_mode)
            return delta
        with stage("mf.sgd", self.timer):
            if self.sgd_mode == "grouped":
                ptr, order = self.grouper.run(pos, n_unique)
                delta = torch.empty((n_unique, c.dim), dtype=torch.float32, device=self.U.device)
                ops.mf_sgd_grouped(self.U, rows, uid_local, rating, ptr, order, c.learning_rate, c.lam, delta)
            else:
                delta = torch.zeros((n_unique, c.dim), dtype=torch.float32, device=self.U.device)
                ops.mf_sgd_pulled(self.U, uid_local, rating, rows, pos, delta, c.learning_rate, c.lam,
                                  self.user_atomic)
        return delta

    def _item_sgd_in_place(self, table: torch.Tensor, staged):
        """PS path, world 1 (``_MFPSWorker``): the tiled SGD of one micro-batch on the
        served shard itself, its push (the rows' summed deltas) added in place."""
        c = self.cfg
        ptr, rec, ev = staged
        if ev is not None:
            torch.cuda.current_stream(self.U.device).wait_event(ev)
        with stage("mf.sgd", self.timer):
            for p in range(self.user_phases):
                ops.mf_sgd_tiled(self.U, table, rec, ptr, 2 * p, self.tile_T, self.tile_R, c.learning_rate, c.lam,
                                 user_mode=self.user_mode)

    def flush(self):
        """Complete the in-flight micro-batch of the pipelined path / bring the
        rotating item blocks back to their PS shards."""
        if self.sgd_mode == "tiled" and self._staged is not None:
            staged, self._staged = self._staged, None
            self._tiled_sgd(staged)
        if self.exchange == "rotate" and not self.rot.at_rest:
            self.rot.home()
            if self.items.touched is not None and self.comm.world == 1:
                self.items.touched |= self._seen
            elif self.items.touched is not None:
                seen = self.comm.all_reduce(self._seen.clone(), op=torch.distributed.ReduceOp.MAX)
                loc = torch.arange(self.items.n_local, device=seen.device)
                self.items.touched |= seen[self.items.global_ids(loc)]
        if self.exchange == "ps":
            self.runtime.pipe.drain()

    # -------------------------------------------------------------- checkpoint
    _AUX = ("_ring", "_ring_cursor", "_known_flag", "_known", "_known_count")

    def aux_state(self) -> dict:
        """Per-rank state besides the tables (``utils.io.Checkpointer``): the
        negative-sampling RNG counter and rings, the update count."""
        st = {"updates": self.updates}
        if self.cfg.negative_sample_rate > 0:
            st["neg_counter"] = self._neg_counter
            st.update({k: getattr(self, k) for k in self._AUX})
        return st

    def load_aux_state(self, st: dict) -> None:
        self.updates = int(st.get("updates", 0))
        if self.cfg.negative_sample_rate > 0:
            self._neg_counter = int(st["neg_counter"])
            for k in self._AUX:
                getattr(self, k).copy_(st[k])

    def set_timer(self, timer) -> None:
        """Attach a ``utils.metrics.StageTimer`` to the model and its PS."""
        self.timer = timer
        self.ps.timer = timer

    def metrics(self) -> dict:
        """Host counters of this rank (ratings, micro-batches, PS pulls / unique keys,
        bytes put on the wire by the all-to-alls and the ring rotation)."""
        m = self.counters.snapshot()
        m.update({f"ps.{k}": v for k, v in self.ps.stats.items()})
        m["bytes_sent.a2a"] = self.comm.bytes_sent
        if self.exchange == "rotate":
            m["bytes_sent.rotation"] = self.rot.bytes_sent
        return m

    @torch.no_grad()
    def sq_err(self, uid_local, iid, rating) -> float:
        """Sum of squared errors of this rank's ratings (items pulled when remote)."""
        self.flush()
        if self.comm.world == 1:
            return float(ops.mf_sq_err(self.U, self.I, uid_local, iid, rating).item())
        vals = self.ps.pull_values(iid)
        e = rating - (self.U[uid_local.long()] * vals).sum(1)
        return float((e.double() ** 2).sum())

    def rmse(self, uid_local, iid, rating) -> float:
        se = self.comm.sum_over_ranks(self.sq_err(uid_local, iid, rating))
        n = self.comm.sum_over_ranks(float(uid_local.numel()))
        return (se / max(n, 1.0)) ** 0.5

    def load_model(self, users=None, items=None) -> None:
        """Warm start (``transformWithDoubleModelLoad``: users are worker-resident,
        items live on the PS): ``users`` / ``items`` = ``(ids, values)`` tensors or
        ``{id: vector}`` dicts (``utils.io.read_factors_text``).  Every rank may pass
        the whole model; each keeps the rows it owns."""
        self.flush()

        def as_t(m):
            if isinstance(m, dict):
                ids = torch.tensor(sorted(m), dtype=torch.int64)
                vals = torch.tensor([list(m[int(i)]) for i in ids.tolist()], dtype=torch.float32)
                return ids, vals.reshape(ids.numel(), -1)
            return m[0].long(), m[1].float()

        if users is not None:
            self.users.load(*as_t(users))
        if items is not None:
            self.items.load(*as_t(items))

    def user_vectors(self):
        ids = self.users.global_ids(torch.arange(self.users.n_local, device=self.U.device))
        return ids, self.U

    def item_vectors(self, only_touched=True):
        self.flush()
        return self.items.dump(only_touched)


class _MFPSWorker(BatchedWorkerLogic):
    """``DistributedMF``'s PS path as a batched worker: pull the items of a
    micro-batch of ``(local user row, item, rating)``, run the model's SGD kernel on
    the answered rows, push the per-item deltas
    (``PSOnlineMatrixFactorizationWorker``, ``M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:41-89``)."""

    def __init__(self, model: "DistributedMF"):
        self.m = model

    def on_recv_batch(self, batch, ps):
        uid_local, iid, rating = batch
        m = self.m
        staged = None
        if m.sgd_mode == "tiled" and m._ps_spec and m.ps.identity_for(iid.numel()):
            # identity plan ahead: bucket by item id now, on the side stream, while an
            # earlier batch's SGD runs (the partition no longer sits on the critical path)
            staged = m._stage_partition(uid_local, iid, rating)
            # the partition marked the rated items: the identity plan's presence flags
            ps.pull(iid, (uid_local, rating, staged), presence=(m._presence[(m._tiler_i - 1) % len(m._tilers)],
                                                                 staged[2]))
            return
        ps.pull(iid, (uid_local, rating, staged))

    def on_pull_recv_batch(self, pulled, ps):
        uid_local, rating, staged = pulled.payload
        m = self.m
        if staged is not None and not getattr(pulled, "identity", False):
            raise RuntimeError("MF PS path: a partition was staged for an identity plan that did not happen")
        if staged is not None and m.cfg.fuse_local_push:
            # world 1, zero-copy identity serve: the pulled rows ARE the shard.  The
            # delta-mode kernel continues every row from "pulled + added so far", which
            # is the row updated in place -- so the kernel adds the push itself
            target = ps.local_push_target(in_place=True)
            if target is not None and target[0].data_ptr() == pulled.rows.data_ptr():
                m._item_sgd_in_place(pulled.rows, staged)
                ps.push_applied()
                return
        ps.push_unique(m._item_deltas(pulled.rows, pulled.pos, pulled.n_unique, uid_local, rating, staged))


@dataclass
class SyntheticRatings:
    """On-device synthetic rating stream of one rank (users of this rank only).

    ``truth_dim > 0`` draws ratings from a hidden low-rank model so RMSE can
    fall; otherwise ratings are U[0, 1) (implicit-feedback-like), which is all
    a throughput run needs.
    """

    num_users: int
    num_items: int
    n: int
    rank: int = 0
    world: int = 1
    seed: int = 1234
    truth_dim: int = 0
    device: str = "cpu"
    uid: torch.Tensor = field(init=False)
    iid: torch.Tensor = field(init=False)
    rating: torch.Tensor = field(init=False)

    def __post_init__(self):
        g = torch.Generator(device=self.device)
        g.manual_seed(self.seed * 1000003 + self.rank)
        n_local_users = (self.num_users - self.rank + self.world - 1) // self.world
        self.uid = torch.randint(0, n_local_users, (self.n,), generator=g, device=self.device, dtype=torch.int32)
        self.iid = torch.randint(0, self.num_items, (self.n,), generator=g, device=self.device, dtype=torch.int32)
        if self.truth_dim > 0:
            gt = torch.Generator(device="cpu")
            gt.manual_seed(self.seed)
            Ut = torch.rand(self.num_users, self.truth_dim, generator=gt) / self.truth_dim ** 0.5
            It = torch.rand(self.num_items, self.truth_dim, generator=gt) / self.truth_dim ** 0.5
            ug = self.rank + self.world * self.uid.long().cpu()
            self.rating = (Ut[ug] * It[self.iid.long().cpu()]).sum(1).to(self.device)
        else:
            self.rating = torch.rand(self.n, generator=g, device=self.device, dtype=torch.float32)

    def batch(self, i: int, size: int):
        s = (i * size) % max(self.n - size + 1, 1)
        return self.uid[s:s + size], self.iid[s:s + size], self.rating[s:s + size]
