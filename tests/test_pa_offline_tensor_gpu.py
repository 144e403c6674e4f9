"""Offline PA apps on the MI355X (PA kernels K10-K12, device shuffle, two-phase replay)."""
import numpy as np
import pytest
import torch

import test_pa_offline_tensor as T
from test_pa import _dict_data, reference_data
from test_pa_reference_scale import F_REF, NNZ_REF

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("paf_type", [0, 1, 2])
def test_offline_binary_gpu(paf_type):
    train, test = _dict_data(400, 30, 1), _dict_data(100, 30, 2)
    preds, _ = T.run_offline(1, train, test, 30, paf_type=paf_type, device=DEV)
    assert len(preds) == len(test) and T._acc(preds, test) >= 0.8


@pytest.mark.parametrize("kind", ["ova", "pb", "ml"])
def test_offline_multiclass_gpu(kind):
    train, test = _dict_data(600, 30, 1, multi=True), _dict_data(100, 30, 2, multi=True)
    preds, n_model = T.run_offline(1, train, test, 30, kind=kind, L=3, paf_type=1, device=DEV)
    assert T._acc(preds, test) >= 0.7 and n_model > 0


def test_offline_binary_reference_scale_gpu():
    ref = reference_data(F_REF, nnz=NNZ_REF)
    train = [({int(k): float(v) for k, v in zip(x.indices.tolist(), x.values.tolist())}, 1 if y else -1)
             for x, y in ref]
    preds, _ = T.run_offline(1, train, train[:20], F_REF, iterations=3, mb=4, device=DEV)
    assert T._acc(preds, train[:20]) >= 0.8
