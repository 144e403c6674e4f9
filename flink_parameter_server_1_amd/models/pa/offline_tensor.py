"""Offline (multi-epoch) PA classification on the tensor engine.

``PABinaryClassificationOffline`` / ``PAMultiClassificationOffline``
(``M/passive/aggressive/classification/binary/PABinaryClassificationOffline.scala:47-387``)
build a two-phase EOF protocol by hand: sources broadcast EOF signs, a
coordinator holds the test data back until the training input ended, a worker
thread replays ``iterations`` (unshuffled) epochs of pulls under an
in-flight limit, waits until every answer was applied, then pulls the test
vectors' weights and predicts (``:107-297``); predictions are logged at close as
``###PS###t;<label>;[k -> v,...]`` (``:353-358``).

Here the same protocol is the tensor engine's end-of-input replay
(``TensorRuntime.execute`` -> ``BatchedWorkerLogic.on_eof``):

1. streaming phase -- every rank buffers its ``("train", csr)`` and ``("test",
   csr)`` micro-batches on the device (no pulls);
2. ``on_eof`` #1 -- the training examples are concatenated and replayed for
   ``iterations`` epochs, each a real device shuffle (``torch.randperm`` on the
   GPU + a CSR row gather, B2 fixed), in micro-batches of ``micro_batch``
   examples: pull the active features, PA step (``ops.pa_binary`` /
   ``ops.pa_multi``, K10-K12), push the summed deltas;
3. the phase ends with the pipeline drained on every rank (all pushes applied:
   the reference's "wait until all answers arrived");
4. ``on_eof`` #2 -- the test micro-batches are replayed unlabelled: pull,
   predict, output ``Left((example ids, labels))``; no push changes the model;
5. ``close`` logs every prediction in the reference's format when INFO logging
   is on for this module.

The model ends on the PS shards (``SimplePSLogicWithClose`` / range-partitioned
``RangePSLogicWithClose``, dumped as ``Right((feature ids, weights))``).
Variants: binary PA / PA-I / PA-II (the reference's ``pafType`` 0 / 1 / 2 with
``pafConst``), OVA multiclass, cost-based PB / ML (B8: the reference's
multiclass app is a copy of the binary one).
"""
from __future__ import annotations

import logging
from typing import Iterable, Iterator, List, Optional

import torch

from ... import ops
from ...api.batched import BatchedWorkerLogic
from ...core.tensor_engine import TensorRuntime
from ...parallel.comm import Comm
from ...ps.device_logics import DeviceRangePSLogicWithClose, DeviceSimplePSLogicWithClose

log = logging.getLogger("flink_parameter_server_1_amd.pa.offline")

PAF_VARIANTS = {0: "PA", 1: "PA-I", 2: "PA-II"}


def _cat_csr(batches: List[tuple], device) -> tuple:
    """One CSR ``(indptr int64, indices int32, values fp32, labels, ids)`` of many."""
    if not batches:
        z = torch.zeros(0, dtype=torch.int64, device=device)
        return (torch.zeros(1, dtype=torch.int64, device=device), z.to(torch.int32), z.float(), z.to(torch.int32), z)
    lens = torch.cat([b[0][1:] - b[0][:-1] for b in batches])
    indptr = torch.zeros(lens.numel() + 1, dtype=torch.int64, device=device)
    indptr[1:] = torch.cumsum(lens, 0)
    return (indptr, torch.cat([b[1] for b in batches]), torch.cat([b[2] for b in batches]),
            torch.cat([b[3] for b in batches]), torch.cat([b[4] for b in batches]))


def shuffle_csr(csr: tuple, gen: torch.Generator) -> tuple:
    """Examples of a CSR batch in a random order, on the device (no host sync:
    the total nnz is known, so the row gather needs no output-size readback)."""
    indptr, idx, val, lab, ids = csr
    B = lab.numel()
    if B == 0:
        return csr
    p = torch.randperm(B, generator=gen, device=lab.device)
    lens = (indptr[1:] - indptr[:-1])[p]
    nptr = torch.zeros_like(indptr)
    nptr[1:] = torch.cumsum(lens, 0)
    nnz = idx.numel()
    off = torch.repeat_interleave(indptr[:-1][p] - nptr[:-1], lens, output_size=nnz) + \
        torch.arange(nnz, device=lab.device)
    return nptr, idx[off], val[off], lab[p], ids[p]


def chunk_csr(csr: tuple, micro_batch: int) -> Iterator[tuple]:
    """Micro-batches of ``micro_batch`` examples (one host read of the boundaries)."""
    indptr, idx, val, lab, ids = csr
    B = lab.numel()
    starts = list(range(0, B, micro_batch)) + [B]
    bounds = indptr[torch.tensor(starts, device=indptr.device)].tolist()
    for k in range(len(starts) - 1):
        s, e = starts[k], starts[k + 1]
        a, b = bounds[k], bounds[k + 1]
        yield (indptr[s:e + 1] - a, idx[a:b], val[a:b], lab[s:e], ids[s:e])


class OfflinePAWorker(BatchedWorkerLogic):
    """The worker of the offline apps (see the module docstring)."""

    def __init__(self, kind: str = "binary", label_count: int = 1, variant: str = "PA", C: float = 1.0,
                 cost: Optional[torch.Tensor] = None, iterations: int = 1, micro_batch: int = 256, seed: int = 0):
        if kind not in ("binary", "ova", "pb", "ml"):
            raise ValueError(kind)
        self.kind, self.L = kind, (1 if kind == "binary" else int(label_count))
        self.variant, self.C, self.cost_host = variant, float(C), cost
        self.iterations, self.micro_batch, self.seed = int(iterations), int(micro_batch), int(seed)
        self.train: List[tuple] = []
        self.test: List[tuple] = []
        self.phase = "stream"
        self.predictions: List[tuple] = []  # (test csr, labels) for the close-time log
        self.epochs_done = 0

    def open(self, ctx):
        self.device = torch.device(ctx.device)
        self.rank = ctx.index_of_this_subtask
        self.cost = None
        if self.kind in ("pb", "ml"):
            c = self.cost_host if self.cost_host is not None else 1.0 - torch.eye(self.L)
            self.cost = c.to(self.device, torch.float32).contiguous()
        self._n_test = 0

    def _as_csr(self, batch, test: bool) -> tuple:
        indptr, indices, values = (t.to(self.device) for t in batch[:3])
        B = indptr.numel() - 1
        if test:
            labels = torch.full((B,), 0 if self.kind == "binary" else -1,
                                dtype=torch.int8 if self.kind == "binary" else torch.int32, device=self.device)
            ids = batch[3].to(self.device).long() if len(batch) > 3 else \
                torch.arange(self._n_test, self._n_test + B, device=self.device)
            self._n_test += B
        else:
            labels = batch[3].to(self.device)
            labels = labels.to(torch.int8 if self.kind == "binary" else torch.int32)
            ids = torch.full((B,), -1, dtype=torch.int64, device=self.device)
        return indptr.long(), indices.to(torch.int32).contiguous(), values.float().contiguous(), labels, ids

    def on_recv_batch(self, batch, ps):
        if self.phase == "stream":  # buffer until the end of input (no pulls)
            tag, csr = batch
            if tag not in ("train", "test"):
                raise ValueError(f"offline PA input must be ('train' | 'test', csr), not {tag!r}")
            (self.train if tag == "train" else self.test).append(self._as_csr(csr, tag == "test"))
            return
        _, csr = batch  # a replayed ("train" | "test", csr) micro-batch
        ps.pull(csr[1], csr)

    def on_pull_recv_batch(self, pulled, ps):
        indptr, _, values, labels, ids = pulled.payload
        rows = pulled.rows.float().contiguous()
        train = self.phase == "train"
        delta = torch.zeros((pulled.n_unique, self.L), dtype=torch.float32, device=rows.device)
        if self.kind == "binary":
            pred, _ = ops.pa_binary(indptr, values, pulled.pos, rows.view(-1), labels, self.variant, self.C,
                                    delta.view(-1))
        else:
            pred, _ = ops.pa_multi(indptr, values, pulled.pos, rows, labels, self.kind, self.variant, self.C,
                                   self.cost, delta)
        if train:
            ps.push_unique(delta)
        else:  # every example of a test batch is unlabelled: no masking, no host sync
            out = pred.to(torch.int64)
            ps.output((ids, out))
            self.predictions.append((pulled.payload, out))

    def on_eof(self, ps) -> Optional[Iterable]:
        if self.phase == "stream":
            self.phase = "train"
            return self._epochs(_cat_csr(self.train, self.device))
        if self.phase == "train":
            self.phase = "predict"
            return [("test", b) for b in self.test]
        return None

    def _epochs(self, csr) -> Iterator:
        gen = torch.Generator(device=self.device)
        gen.manual_seed(self.seed * 1000003 + self.rank)
        for _ in range(self.iterations):
            for b in chunk_csr(shuffle_csr(csr, gen), self.micro_batch):
                yield ("train", b)
            self.epochs_done += 1

    def close(self, ps=None):
        if not log.isEnabledFor(logging.INFO):
            return
        for (indptr, idx, val, _, _), labels in self.predictions:
            ip, ix, vx, lb = indptr.tolist(), idx.tolist(), val.tolist(), labels.tolist()
            for j, lab in enumerate(lb):
                feats = sorted(zip(ix[ip[j]:ip[j + 1]], vx[ip[j]:ip[j + 1]]))
                log.info("###PS###t;%s;[%s]", lab, ",".join(f"{k} -> {v}" for k, v in feats))


def pa_classification_offline_tensor(source: Iterable, feature_count: int, *, kind: str = "binary",
                                     label_count: int = 1, variant: str = "PA", C: float = 1.0, iterations: int = 1,
                                     micro_batch: int = 256, range_partitioning: bool = False,
                                     cost: Optional[torch.Tensor] = None, seed: int = 0, comm: Optional[Comm] = None,
                                     staleness: int = 0, output_sink=None) -> list:
    """This rank's part of the offline PA app: ``source`` yields ``("train", (indptr,
    indices, values, labels))`` and ``("test", (indptr, indices, values[, ids]))``
    micro-batches (binary labels +-1, multiclass 0..L-1).  Returns this rank's
    outputs: ``Left((test ids, predicted labels))`` and, at close,
    ``Right((feature ids, weights))``."""
    L = 1 if kind == "binary" else int(label_count)
    if range_partitioning:
        logic = DeviceRangePSLogicWithClose(feature_count, L, init=("zeros",))
    else:
        logic = DeviceSimplePSLogicWithClose(feature_count, L, init=("zeros",), partition="hash")
    worker = OfflinePAWorker(kind, L, variant, C, cost, iterations, micro_batch, seed)
    rt = TensorRuntime(comm, staleness=staleness, output_sink=output_sink)
    return rt.execute(source, worker, logic)


def pa_binary_classification_offline_tensor(training: Iterable, test: Iterable, feature_count: int, *,
                                            iterations: int, paf_type: int = 0, paf_const: float = 1.0,
                                            **kw) -> list:
    """``paBinaryClassificationOffline``'s knobs (``pafType`` 0 / 1 / 2, ``pafConst``)
    over this rank's ``training`` / ``test`` CSR micro-batches."""
    src = [("train", b) for b in training] + [("test", b) for b in test]
    return pa_classification_offline_tensor(src, feature_count, kind="binary", variant=PAF_VARIANTS[paf_type],
                                            C=paf_const, iterations=iterations, **kw)


def pa_multi_classification_offline_tensor(training: Iterable, test: Iterable, feature_count: int,
                                           label_count: int, *, iterations: int, kind: str = "ova",
                                           paf_type: int = 0, paf_const: float = 1.0, **kw) -> list:
    """The multiclass app (OVA by default; ``kind="pb"`` / ``"ml"``: cost based)."""
    src = [("train", b) for b in training] + [("test", b) for b in test]
    return pa_classification_offline_tensor(src, feature_count, kind=kind, label_count=label_count,
                                            variant=PAF_VARIANTS[paf_type], C=paf_const, iterations=iterations,
                                            **kw)
