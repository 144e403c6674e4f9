"""Sparse pairwise-embedding training on a huge sharded table (BASELINE config #5).

Config #5 of the north star is "100B-param embedding table sharded across
8 x 288 GB HBM (PS capacity / bounded-staleness stress)".  The reference keeps
every parameter in a Flink operator's heap map (``M/server/SimplePSLogic.scala``,
``RangePSLogicWithClose`` for dense id spaces, ``M/server/RangePSLogicWithClose.scala:51-62``)
and bounds asynchrony with ``pullLimit`` (``M/WorkerLogic.scala:176-225``).  Here:

* the table is a range-partitioned ``ShardedTable`` (``|id| // ceil(F/P)``):
  100e9 fp32 parameters at dim 64 = 1.5625e9 rows, 50 GB per GPU over 8
  (Adagrad doubles it to 100 GB -- still well inside 288 GB);
* each micro-batch is a set of (a, b, label) id pairs with power-law id
  popularity; both rows are pulled through the deduplicating ``TensorPS``
  (hashed claim map: the id space is far above the dense-map limit);
* the fused ``pair_sgd_pulled`` kernel scores ``<e_a, e_b>`` (logistic or
  squared loss) and accumulates per-unique-row deltas;
* ``BoundedStalenessPipeline`` keeps up to ``staleness`` later pulls in flight
  before a push is applied.

Synthetic task: ids belong to ``clusters`` classes (``id % clusters``); a
positive pair shares the class, a negative pair is uniform.  Learnable, cheap
to generate on the device, and no host-side truth table is needed at 1e9+ ids.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from ... import ops
from ...parallel.comm import Comm
from ...parallel.staleness import BoundedStalenessPipeline
from ...parallel.table import ShardedTable
from ...parallel.tensor_ps import TensorPS
from ...utils.tracing import stage

_WIRE = {"fp32": torch.float32, "bf16": torch.bfloat16}
MAX_IDS = (1 << 31) - 1  # keys travel as int32


@dataclass
class PairEmbeddingConfig:
    num_ids: int = 1_562_500_000       # 100e9 parameters at dim 64
    dim: int = 64
    learning_rate: float = 0.05
    loss: str = "logistic"             # or "squared"
    optimizer: str = "add"             # PS update rule: "add" (SGD deltas) or "adagrad"
    staleness: int = 1                 # pushes a pull may miss (0 = synchronous)
    partition: str = "range"
    init_scale: float = 0.5            # U[-s, s) / sqrt(dim)
    wire_dtype: str = "fp32"
    seed: int = 0

    @property
    def num_params(self) -> int:
        return self.num_ids * self.dim


class DistributedPairEmbedding:
    def __init__(self, cfg: PairEmbeddingConfig, comm: Optional[Comm] = None, track_touched: bool = False):
        if cfg.num_ids > MAX_IDS:
            raise ValueError(f"num_ids {cfg.num_ids} exceeds the int32 key space; raise dim instead")
        if cfg.optimizer not in ("add", "adagrad"):
            raise ValueError(cfg.optimizer)
        self.cfg = cfg
        self.comm = comm or Comm()
        s = cfg.init_scale / cfg.dim ** 0.5
        self.table = ShardedTable(cfg.num_ids, cfg.dim, self.comm.rank, self.comm.world, cfg.partition,
                                  ("uniform", -s, s), cfg.seed, self.comm.device, cfg.optimizer,
                                  track_touched=track_touched)
        self.ps = TensorPS(self.table, self.comm, _WIRE[cfg.wire_dtype])
        # Adagrad: the PS applies w -= lr * g / sqrt(sum g^2); the kernel then
        # emits the raw gradient (-(label - p) * e_other), i.e. kernel lr = -1.
        self._kernel_lr = cfg.learning_rate if cfg.optimizer == "add" else -1.0
        self._ps_lr = cfg.learning_rate if cfg.optimizer == "adagrad" else 0.0
        self.pipe = BoundedStalenessPipeline(self.ps, self._compute, cfg.staleness, lr=self._ps_lr)
        self.pairs_seen = 0
        self.rows_pushed = 0

    def _compute(self, rows, plan, payload):
        n_pairs, labels, with_loss = payload
        delta = torch.zeros((plan.n_unique, self.cfg.dim), dtype=torch.float32, device=rows.device)
        pos = plan.pos
        with stage("pairs.step", None):
            loss = ops.pair_sgd_pulled(rows, pos[:n_pairs], pos[n_pairs:], labels, delta, self._kernel_lr,
                                       self.cfg.loss, with_loss)
        self.rows_pushed += plan.n_unique
        return delta, (loss, n_pairs)

    def step(self, a: torch.Tensor, b: torch.Tensor, labels: torch.Tensor, with_loss: bool = False):
        """Submit one micro-batch; returns ``[(loss_sum or None, n_pairs), ...]``
        for the batches whose push completed during this call."""
        keys = torch.cat([a.to(torch.int32), b.to(torch.int32)])
        self.pairs_seen += a.numel()
        return self.pipe.submit(keys, (a.numel(), labels.to(torch.float32).contiguous(), with_loss))

    def flush(self):
        return self.pipe.drain()

    def mean_loss(self, a, b, labels) -> float:
        """Loss of a batch against the current table (no update; flushes first)."""
        self.flush()
        rows, plan = self.ps.pull(torch.cat([a.to(torch.int32), b.to(torch.int32)]))
        delta = torch.zeros((plan.n_unique, self.cfg.dim), dtype=torch.float32, device=rows.device)
        loss = ops.pair_sgd_pulled(rows, plan.pos[:a.numel()], plan.pos[a.numel():],
                                   labels.to(torch.float32).contiguous(), delta, 0.0, self.cfg.loss, True)
        tot = self.comm.sum_over_ranks(float(loss.sum()))
        n = self.comm.sum_over_ranks(float(a.numel()))
        return tot / max(n, 1.0)


def cluster_of(ids: torch.Tensor, clusters: int) -> torch.Tensor:
    return ids % clusters


def synthetic_pairs(num_ids: int, n: int, seed: int = 0, step: int = 0, device="cpu", zipf: float = 1.5,
                    clusters: int = 16, pos_frac: float = 0.5):
    """``(a, b, label)`` with power-law id popularity (``u ** zipf`` scaled to the
    id space, scrambled by a multiplicative hash so hot ids spread over shards)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed * 1_000_003 + step)

    def draw(m):
        u = torch.rand(m, generator=g, device=device, dtype=torch.float64)
        rank = (u ** zipf * num_ids).long().clamp_(max=num_ids - 1)
        return (rank * 2654435761) % num_ids

    a = draw(n)
    b = draw(n)
    label = (torch.rand(n, generator=g, device=device) < pos_frac)
    # positives: move b into a's cluster (stay inside the id space)
    same = b - cluster_of(b, clusters) + cluster_of(a, clusters)
    same = torch.where(same >= num_ids, same - clusters, same)
    b = torch.where(label, same, b)
    return a.to(torch.int32), b.to(torch.int32), label.to(torch.float32)
