"""Passive-Aggressive worker for the tensor engine (``core.tensor_engine``).

``PassiveAggressiveParameterServer.transformGeneric``'s worker
(``M/passive/aggressive/PassiveAggressiveParameterServer.scala:283-338``) on
micro-batches: the worker pulls every active feature of its examples (one pull
per micro-batch, duplicates deduplicated by the engine), runs the PA step of
every example on the pulled weights (K10-K12: ``ops.pa_binary`` /
``ops.pa_multi``, one wave per example, per-feature deltas summed per unique
feature in the kernel) and pushes the summed deltas (``push_unique``).
Unlabelled examples (binary label 0, multiclass -1) are predicted and emitted as
``Left((example ids, labels))`` (an ``api.batched.MaskedPair``: compacted when
read, so the step issues no host sync); the PS logic (range partitioned
``RangePSLogicWithClose`` or hash ``SimplePSLogicWithClose``, ``:262-281``) dumps
the model at close as ``Right((feature ids, weights))``.

Batches are CSR tuples ``(indptr int64 [B+1], indices int32 [nnz], values fp32
[nnz], labels [B])`` with an optional fifth entry, the example ids for the
prediction output (default: the example's position in the stream of this rank).
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch

from ... import ops
from ...api.batched import BatchedWorkerLogic, MaskedPair
from ...core.tensor_engine import TensorRuntime
from ...parallel.comm import Comm
from ...ps.device_logics import DeviceRangePSLogicWithClose, DeviceSimplePSLogicWithClose


class PAWorker(BatchedWorkerLogic):
    def __init__(self, kind: str = "binary", label_count: int = 1, variant: str = "PA", C: float = 1.0,
                 cost: Optional[torch.Tensor] = None, with_loss: bool = False, emit_predictions: bool = True):
        if kind not in ("binary", "ova", "pb", "ml"):
            raise ValueError(kind)
        self.kind, self.L = kind, (1 if kind == "binary" else int(label_count))
        self.variant, self.C, self.cost_host = variant, float(C), cost
        self.with_loss, self.emit_predictions = with_loss, emit_predictions
        self.last = None          # (predictions [B], loss) of the latest micro-batch
        self.examples = 0
        self._seen = 0
        #: apply the push in the kernel when the PS offers a local target (world 1)
        self.fuse_local_push = True

    def open(self, ctx):
        self.device = torch.device(ctx.device)
        self.cost = None
        if self.kind in ("pb", "ml"):
            c = self.cost_host if self.cost_host is not None else 1.0 - torch.eye(self.L)
            self.cost = c.to(self.device, torch.float32).contiguous()

    def on_recv_batch(self, batch, ps):
        indptr, indices, values, labels = (t.to(self.device) for t in batch[:4])
        ids = batch[4].to(self.device) if len(batch) > 4 else None
        ps.pull(indices, (indptr, values.float().contiguous(), labels, ids))

    def on_pull_recv_batch(self, pulled, ps):
        indptr, values, labels, ids = pulled.payload
        rows = pulled.rows.float().contiguous()
        # one rank owns every feature: the kernel adds the push to the table itself
        # (reading the pulled snapshot), no delta buffer, zeroing or apply pass
        target = ps.local_push_target() if self.fuse_local_push else None
        if target is not None:
            delta, wmap = target
        else:
            delta = torch.zeros((pulled.n_unique, self.L), dtype=torch.float32, device=rows.device)
            wmap = None
        if self.kind == "binary":
            pred, loss = ops.pa_binary(indptr, values, pulled.pos, rows.view(-1), labels, self.variant, self.C,
                                       delta.view(-1), self.with_loss, wmap=wmap)
        else:
            pred, loss = ops.pa_multi(indptr, values, pulled.pos, rows, labels, self.kind, self.variant, self.C,
                                      self.cost, delta, self.with_loss, wmap=wmap)
        if target is not None:
            ps.push_applied()
        else:
            ps.push_unique(delta)
        B = indptr.numel() - 1
        if self.emit_predictions:  # the unlabelled examples' predictions, compacted by the consumer (no sync)
            if ids is None:
                ids = torch.arange(self._seen, self._seen + B, device=labels.device)
            ps.output(MaskedPair(ids, pred, labels == (0 if self.kind == "binary" else -1)))
        self._seen += B
        self.examples += B
        self.last = (pred, loss)


def transform_pa_tensor(batches: Iterable, feature_count: int, kind: str = "binary", label_count: int = 1,
                        variant: str = "PA", C: float = 1.0, range_partitioning: bool = True, model=None,
                        cost: Optional[torch.Tensor] = None, comm: Optional[Comm] = None, staleness: int = 0,
                        wire: str = "fp32", worker_parallelism: Optional[int] = None,
                        ps_parallelism: Optional[int] = None):
    """``transformBinary`` / ``transformMulticlass`` on the tensor engine (this rank's
    part; ``batches`` = this rank's CSR micro-batches).  ``model`` = this rank's
    ``(feature, weight(s))`` warm-start records (``transformWithModelLoad``).
    ``ps_parallelism`` P <= ranks: the model lives in P shards (``rangePartitionerPS``
    over P, ``PassiveAggressiveParameterServer.scala:372-384``) on ranks 0..P-1."""
    L = 1 if kind == "binary" else label_count
    Logic = DeviceRangePSLogicWithClose if range_partitioning else DeviceSimplePSLogicWithClose
    logic = Logic(feature_count, L, init=("zeros",), wire_dtype=wire) if range_partitioning else \
        Logic(feature_count, L, init=("zeros",), partition="hash", wire_dtype=wire)
    rt = TensorRuntime(comm, staleness=staleness, worker_parallelism=worker_parallelism,
                       ps_parallelism=ps_parallelism)
    return rt.execute(batches, PAWorker(kind, L, variant, C, cost), logic, model=model)
