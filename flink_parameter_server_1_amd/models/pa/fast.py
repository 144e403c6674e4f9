"""Passive-Aggressive on the tensor engine (BASELINE config #4: 1B-dim sparse features).

Same learning rules and data flow as ``PassiveAggressiveParameterServer``
(``M/passive/aggressive/PassiveAggressiveParameterServer.scala:239-370``):
a worker pulls the weights of every active feature of its examples, computes
the PA step and pushes per-feature deltas that the PS adds; the PS table is
range-partitioned by default (``rangePartitionerPS``, ``:372-384``).  Here a
micro-batch of examples travels as CSR tensors; the features are
deduplicated and pulled with one all-to-all (``TensorPS``), one wave per
example runs the PA step on the GPU (``ops.pa_binary`` / ``ops.pa_multi``,
K10-K12), and the per-unique-feature deltas are pushed back.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ... import ops
from ...core.tensor_engine import TensorRuntime
from ...parallel.comm import Comm
from ...parallel.table import ShardedTable
from ...parallel.tensor_ps import TensorPS
from ...ps.device_logics import DeviceRangePSLogicWithClose, DeviceSimplePSLogicWithClose
from .batched import PAWorker
from ...utils.tracing import stage

_WIRE = {"fp32": torch.float32, "bf16": torch.bfloat16}


@dataclass
class PAConfig:
    feature_count: int
    kind: str = "binary"          # binary | ova | pb | ml
    label_count: int = 1
    variant: str = "PA"           # PA | PA-I | PA-II (binary / ova)
    aggressiveness: float = 1.0   # C
    partition: str = "range"      # range | hash
    wire_dtype: str = "fp32"
    local_direct: bool = True     # W = 1: the PA kernel reads / atomically updates the table in place
    #: the most feature requests (nnz) a rank submits per micro-batch: fixed-shape PS
    #: plans (``TensorPS.capacity``: no split sizes on the host, capturable steps)
    capacity: Optional[int] = None
    fuse_local_push: bool = True  # W = 1 PS path: the kernel adds its pushes into the table (no delta buffer)
    #: PS path: micro-batches in flight (the reference's asynchronous pulls under a pull
    #: limit, ``PassiveAggressiveParameterServer.scala:283-338``; ``tensor_engine.
    #: staleness_for_pull_limit``): 1 = the pulls of batch k+1 overlap batch k's step and
    #: its pushes (the row all-to-alls hide behind compute at N > 1); ``flush()`` drains
    staleness: int = 0
    #: PS path at N > 1: serve / apply on a second stream (None: the pipeline's default where
    #: it applies); False (default): the interleaved single-stream schedule (measured faster)
    owner_stream: Optional[bool] = False


class DistributedPA:
    def __init__(self, cfg: PAConfig, comm: Optional[Comm] = None, cost: Optional[torch.Tensor] = None):
        self.cfg = cfg
        self.comm = comm or Comm()
        self.L = 1 if cfg.kind == "binary" else cfg.label_count
        if self.L > 64:
            raise ValueError("multiclass kernels keep the classes on the 64 lanes: label_count <= 64")
        W, r, dev = self.comm.world, self.comm.rank, self.comm.device
        # untouched features hold the -0.0 sentinel (ShardedTable touch_sentinel): the
        # close-time dump of touched features needs no byte-mark pass per micro-batch
        self.table = ShardedTable(cfg.feature_count, self.L, r, W, cfg.partition, ("zeros",), 0, dev,
                                  optimizer="add", touch_sentinel=True)
        self.ps = TensorPS(self.table, self.comm, _WIRE[cfg.wire_dtype])
        if cfg.kind in ("pb", "ml"):
            if cost is None:
                cost = 1.0 - torch.eye(self.L)
            self.cost = cost.to(dev, torch.float32).contiguous()
        else:
            self.cost = None
        self.examples = 0
        # the pull / push path is the public batched API on the tensor engine: a
        # PAWorker + the range / hash WithClose device logic over this model's shard
        Logic = DeviceRangePSLogicWithClose if cfg.partition == "range" else DeviceSimplePSLogicWithClose
        kw = dict(table=self.table, ps=self.ps)
        logic = Logic(cfg.feature_count, self.L, **kw) if cfg.partition == "range" else \
            Logic(cfg.feature_count, self.L, partition=cfg.partition, **kw)
        self.worker = PAWorker(cfg.kind, self.L, cfg.variant, cfg.aggressiveness, self.cost, emit_predictions=False)
        self.worker.fuse_local_push = cfg.fuse_local_push
        # no owner stream: PA's worker side is a chain of short latency-bound kernels that
        # a concurrent 4M-row atomic apply slows 2-5x; the interleaved schedule hides the
        # transfers on one stream instead (profiles/r6_ps_paths_hot_owner.md)
        self.runtime = TensorRuntime(self.comm, staleness=cfg.staleness, capacity=cfg.capacity,
                                     owner_stream=cfg.owner_stream).start(self.worker, logic)
        self.timer = None  # utils.metrics.StageTimer (optional)

    @property
    def _direct(self) -> bool:
        return (self.cfg.local_direct and self.comm.world == 1 and self.table.optimizer == "add"
                and self.table.partition in ("range", "hash"))

    def _run(self, indptr, indices, values, labels, train: bool, with_loss=False):
        c = self.cfg
        if self._direct:
            # one shard holding every feature (local row = feature id): the kernel reads
            # the weights of each example's features and adds its deltas in place -- no
            # dedup, gather, delta buffer or apply pass (asynchronous like the
            # reference's per-feature pull / push interleaving)
            w = self.table.weight
            idx = indices.to(device=w.device, dtype=torch.int32).contiguous()
            # train steps pull (the reference creates a feature's entry on its first pull):
            # the kernel flips the -0.0 sentinel of first-pulled features as it reads them
            flip = w if train else None
            with stage("pa.step", self.timer):
                if c.kind == "binary":
                    pred, loss = ops.pa_binary(indptr, values, idx, w.view(-1), labels, c.variant,
                                               c.aggressiveness, w.view(-1), with_loss,
                                               flip=None if flip is None else flip.view(-1))
                else:
                    pred, loss = ops.pa_multi(indptr, values, idx, w, labels, c.kind, c.variant, c.aggressiveness,
                                              self.cost, w, with_loss, flip=flip)
            if train:
                self.examples += indptr.numel() - 1
            return pred, loss
        # one micro-batch through the engine (staleness 0: done inside submit; staleness s:
        # the batch submitted s calls earlier completes); a predict-only call drains the
        # pipeline first and skips the push round (collective: every rank predicts)
        if not train:
            self.flush()
        self.worker.with_loss = with_loss
        self.worker.pushes = train
        with stage("pa.step", self.timer):
            self.runtime.submit((indptr, indices, values, labels))
        if not train:
            self.flush()  # the predictions of THIS batch
        if train:
            self.examples += indptr.numel() - 1
        return self.worker.last

    def train_step(self, indptr, indices, values, labels, with_loss=False):
        """Labels: binary +1/-1 (int8, 0 = predict only); multiclass class id (int32, -1 = predict only).

        Returns ``(predictions, loss)`` of the micro-batch that COMPLETES during this call:
        this one at ``staleness == 0`` (and on the local-direct path); with the PS path's
        pipeline (``staleness = s > 0``) the batch submitted ``s`` calls earlier -- ``None``
        for the first ``s`` calls -- and ``with_loss`` applies to that completing batch
        (``flush()`` completes the rest; ``predict`` drains first and returns its own)."""
        return self._run(indptr, indices, values, labels, True, with_loss)

    def predict(self, indptr, indices, values):
        B = indptr.numel() - 1
        dev = values.device
        y = (torch.zeros(B, dtype=torch.int8, device=dev) if self.cfg.kind == "binary"
             else torch.full((B,), -1, dtype=torch.int32, device=dev))
        return self._run(indptr, indices, values, y, False)[0]

    def flush(self) -> None:
        """Complete every micro-batch in flight (their pushes applied)."""
        if self.runtime.pipe is not None:
            self.runtime.pipe.drain()

    def dump(self, only_touched=True):
        self.flush()
        return self.table.dump(only_touched)


def synthetic_sparse_batch(B: int, nnz: int, feature_count: int, seed: int, step: int, label_count: int = 1,
                           device="cpu", zipf: float = 1.0):
    """CSR batch with labels from a hidden sparse linear model (hash-defined per feature),
    so a PA learner has signal.  Features drawn ``F * u^(1+zipf)`` (skewed toward low ids)."""
    g = torch.Generator(device=device)
    g.manual_seed((seed * 1_000_003 + step) & 0x7FFFFFFF)
    # fp64 draws: an fp32 u has a 24-bit mantissa, so F * u at F = 1e9 reached only ~2^24
    # ids, nearly all multiples of 64 -- hash sharding (id % N) then sent ~95 % of the keys
    # to shard 0 (round 6, profiles/r6_ps_paths_hot_owner.md)
    u = torch.rand(B * nnz, generator=g, device=device, dtype=torch.float64)
    idx = torch.clamp((u ** (1.0 + zipf) * feature_count).long(), max=feature_count - 1)
    vals = torch.rand(B * nnz, generator=g, device=device) + 0.1
    indptr = torch.arange(0, B * nnz + 1, nnz, dtype=torch.int64, device=device)
    # hidden model: per-feature class preferences from a hash of the id
    from ...ops.reference import fmix32

    h = fmix32((idx & 0xFFFFFFFF) ^ 0x5BD1E995)
    if label_count == 1:
        s = ((h & 0xFFFF).float() / 65535.0 - 0.5)
        margin = torch.zeros(B, device=device).index_add_(0, torch.arange(B, device=device).repeat_interleave(nnz),
                                                          vals * s)
        labels = torch.where(margin > 0, 1, -1).to(torch.int8)
    else:
        cls = (h % label_count)
        scores = torch.zeros(B, label_count, device=device)
        scores.index_put_((torch.arange(B, device=device).repeat_interleave(nnz), cls), vals, accumulate=True)
        labels = torch.argmax(scores, 1).to(torch.int32)
    return indptr, idx.to(torch.int32), vals, labels
