"""Offline PA apps on the tensor engine (``models/pa/offline_tensor.py``): the
two-phase train-epochs-then-predict protocol of ``PABinaryClassificationOffline``
(``M/passive/aggressive/classification/binary/PABinaryClassificationOffline.scala:47-387``)
-- accuracy against the per-record app, gloo W = 1 / 3; device shuffle; CSR
helpers."""
import numpy as np
import pytest
import torch

from dist_utils import run_ranks
from flink_parameter_server_1_amd.core.messages import Left, Right
from flink_parameter_server_1_amd.models.pa.offline_tensor import chunk_csr, shuffle_csr
from test_pa import _dict_data, reference_data
from test_pa_reference_scale import F_REF, NNZ_REF


def _csr_dicts(examples, labels=True, multi=False):
    indptr, idx, val, lab = [0], [], [], []
    for x, y in examples:
        for k, v in sorted(x.items()):
            idx.append(k)
            val.append(v)
        indptr.append(len(idx))
        lab.append(y)
    out = (torch.tensor(indptr, dtype=torch.int64), torch.tensor(idx, dtype=torch.int32),
           torch.tensor(val, dtype=torch.float32))
    return out + ((torch.tensor(lab, dtype=torch.int32 if multi else torch.int8),) if labels else ())


def _offline_rank(rank, world, train, test, F, kind, L, paf_type, iterations, mb, device=None):
    from flink_parameter_server_1_amd.models.pa.offline_tensor import (pa_binary_classification_offline_tensor,
                                                                       pa_multi_classification_offline_tensor)
    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm(device=device) if device is not None else Comm()
    tr = train[rank::world]  # rebalance: round-robin over the workers
    te_idx = list(range(rank, len(test), world))
    tr_b = [_csr_dicts(tr[s:s + mb], multi=kind != "binary") for s in range(0, len(tr), mb)]
    te_b = []
    for s in range(0, len(te_idx), mb):
        sel = te_idx[s:s + mb]
        te_b.append(_csr_dicts([(test[j][0], 0) for j in sel], labels=False) + (torch.tensor(sel),))
    if kind == "binary":
        out = pa_binary_classification_offline_tensor(tr_b, te_b, F, iterations=iterations, paf_type=paf_type,
                                                      paf_const=1.0, micro_batch=mb, seed=3, comm=comm)
    else:
        out = pa_multi_classification_offline_tensor(tr_b, te_b, F, L, iterations=iterations, paf_type=paf_type,
                                                     paf_const=1.0, micro_batch=mb, seed=3, comm=comm)
    preds = {}
    for e in out:
        if isinstance(e, Left):
            for i, y in zip(e.value[0].tolist(), e.value[1].tolist()):
                preds[int(i)] = int(y)
    n_model = sum(e.value[0].numel() for e in out if isinstance(e, Right))
    return preds, n_model


def run_offline(world, train, test, F, kind="binary", L=1, paf_type=0, iterations=5, mb=16, device=None):
    args = (train, test, F, kind, L, paf_type, iterations, mb, device)
    res = run_ranks(_offline_rank, world, *args) if world > 1 else [_offline_rank(0, 1, *args)]
    preds = {}
    for p, _ in res:
        preds.update(p)
    return preds, sum(n for _, n in res)


def _acc(preds, test):
    return np.mean([preds[j] == y for j, (_, y) in enumerate(test)])


@pytest.mark.parametrize("world", [1, 3])
@pytest.mark.parametrize("paf_type", [0, 1, 2])
def test_offline_binary_tensor_matches_per_record_accuracy(world, paf_type):
    from flink_parameter_server_1_amd.core.messages import Left as L_
    from flink_parameter_server_1_amd.models.pa.offline import pa_binary_classification_offline

    train, test = _dict_data(400, 30, 1), _dict_data(100, 30, 2)
    preds, _ = run_offline(world, train, test, 30, paf_type=paf_type)
    assert len(preds) == len(test)
    acc = _acc(preds, test)
    out = pa_binary_classification_offline(train, [x for x, _ in test], worker_parallelism=2, ps_parallelism=2,
                                           iterations=5, paf_type=paf_type, paf_const=1, pull_limit=100, seed=0)
    ref = {tuple(sorted(v.items())): lab for v, lab in (e.value for e in out if isinstance(e, L_))}
    acc_ref = np.mean([ref[tuple(sorted(x.items()))] == y for x, y in test])
    assert acc >= 0.8 and acc >= acc_ref - 0.05, (acc, acc_ref)


@pytest.mark.parametrize("kind", ["ova", "pb", "ml"])
def test_offline_multiclass_tensor(kind):
    train, test = _dict_data(600, 30, 1, multi=True), _dict_data(100, 30, 2, multi=True)
    preds, n_model = run_offline(3, train, test, 30, kind=kind, L=3, paf_type=1)
    assert _acc(preds, test) >= 0.7 and n_model > 0


def test_offline_binary_tensor_reference_scale():
    """The reference test's data (500k dims, ~10k nnz, 80 vectors), trained offline
    for 3 epochs at W = 3, predicting its first 20 training vectors."""
    ref = reference_data(F_REF, nnz=NNZ_REF)
    train = [({int(k): float(v) for k, v in zip(x.indices.tolist(), x.values.tolist())}, 1 if y else -1)
             for x, y in ref]
    preds, _ = run_offline(3, train, train[:20], F_REF, iterations=3, mb=4)
    assert _acc(preds, train[:20]) >= 0.8


def test_shuffle_and_chunk_csr_keep_every_example():
    g = torch.Generator().manual_seed(0)
    lens = torch.randint(0, 5, (37,))
    indptr = torch.zeros(38, dtype=torch.int64)
    indptr[1:] = torch.cumsum(lens, 0)
    nnz = int(indptr[-1])
    csr = (indptr, torch.arange(nnz, dtype=torch.int32), torch.arange(nnz).float(), torch.arange(37),
           torch.arange(37) + 100)
    sh = shuffle_csr(csr, g)
    assert sorted(sh[3].tolist()) == list(range(37)) and not torch.equal(sh[3], csr[3])
    for j, e in enumerate(sh[3].tolist()):  # every example keeps its own features
        assert sh[1][sh[0][j]:sh[0][j + 1]].tolist() == csr[1][indptr[e]:indptr[e + 1]].tolist()
    chunks = list(chunk_csr(sh, 8))
    assert [c[3].numel() for c in chunks] == [8, 8, 8, 8, 5]
    assert torch.equal(torch.cat([c[1] for c in chunks]), sh[1])
