"""Passive-Aggressive — port of T/passive/aggressive/PassiveAggressiveParameterServerTest.scala
(scaled: 100k dims, ~2k nnz instead of 500k / 10k, same generator), plus OVA / cost-based /
model-load tests the reference does not have."""
import numpy as np
import pytest

from flink_parameter_server_1_amd.core.messages import Left, Right, left_values, right_values
from flink_parameter_server_1_amd.models.mf.core import JavaRandom
from flink_parameter_server_1_amd.models.pa.algorithms import (PassiveAggressiveBinaryAlgorithm,
                                                               PassiveAggressiveCostBased,
                                                               PassiveAggressiveOneVersusAll)
from flink_parameter_server_1_amd.models.pa.server import (binary_accuracy, multi_accuracy, transform_binary,
                                                           transform_multiclass, transform_multiclass_with_long_id)
from flink_parameter_server_1_amd.models.pa.sparse import SparseVector, VectorBuilder


def reference_data(feature_count=100_000, nnz=2000, n_train=80, seed=50):
    """Same construction as the reference test (java.util.Random(50), VectorBuilder sums duplicates)."""
    r = JavaRandom(seed)

    def vec():
        b = VectorBuilder(feature_count)
        for _ in range(nnz + 1):
            b.add(r.next_int(feature_count), r.next_double())
        return b.to_sparse_vector()

    train = []
    for _ in range(n_train):
        v = vec()
        train.append((v, (r._next(1) & 1) != 0))
    return train


def _model_from_stream(out, feature_count):
    w = np.zeros(feature_count)
    for fid, val in right_values(out):
        w[fid] = val
    return w


@pytest.mark.parametrize("range_partitioning", [True, False])
def test_binary_pa_accuracy(range_partitioning):
    F = 100_000
    train = reference_data(F)
    out = transform_binary(None, input_source=[Left(x) for x in train], worker_parallelism=3, ps_parallelism=3,
                           passive_aggressive_method=PassiveAggressiveBinaryAlgorithm.build_pa(), pull_limit=10000,
                           feature_count=F, range_partitioning=range_partitioning)
    w = _model_from_stream(out, F)
    acc = binary_accuracy(w, train[:20], PassiveAggressiveBinaryAlgorithm.build_pa())
    assert acc >= 80, acc


@pytest.mark.parametrize("build", [PassiveAggressiveBinaryAlgorithm.build_pa,
                                   lambda: PassiveAggressiveBinaryAlgorithm.build_pai(0.5),
                                   lambda: PassiveAggressiveBinaryAlgorithm.build_paii(0.5)])
def test_binary_variants_tau(build):
    m = build()
    x = SparseVector([1, 3], [1.0, 2.0], 5)
    d = dict(m.delta(x, {1: 0.0, 3: 0.0}, True))
    n = 5.0
    loss = 1.0
    tau = {"PA": loss / n, "PA-I": min(0.5, loss / n), "PA-II": loss / (n + 1 / (2 * 0.5))}[m.variant]
    assert d[1] == pytest.approx(tau) and d[3] == pytest.approx(2 * tau)
    assert m.delta(x, {1: 5.0, 3: 5.0}, True) == []  # margin >= 1: passive


def test_binary_predictions_and_model_load():
    F = 50
    model = [(i, 1.0 if i < 25 else -1.0) for i in range(F)]
    tests = [Right((SparseVector([0, 1], [1.0, 1.0], F), SparseVector([0, 1], [1.0, 1.0], F))),
             Right((SparseVector([30], [1.0], F), SparseVector([30], [1.0], F)))]
    out = transform_binary(model, input_source=tests, worker_parallelism=2, ps_parallelism=2,
                           passive_aggressive_method=PassiveAggressiveBinaryAlgorithm.build_pa(), pull_limit=100,
                           feature_count=F, range_partitioning=True)
    preds = {int(v.indices[0]): lab for v, lab in left_values(out)}
    assert preds == {0: True, 30: False}


def _multi_data(n, F, L, seed):
    centers = np.random.default_rng(0).normal(size=(L, F))
    rng = np.random.default_rng(seed)
    data = []
    for _ in range(n):
        c = int(rng.integers(L))
        idx = np.sort(rng.choice(F, size=12, replace=False))
        vals = centers[c, idx] + 0.1 * rng.normal(size=12)
        data.append((SparseVector(idx, vals, F), c))
    return data


@pytest.mark.parametrize("method", ["ova", "ova1", "ova2", "pb", "ml"])
def test_multiclass_learns(method):
    F, L = 40, 3
    cost = lambda y, q: 0.0 if y == q else 1.0  # noqa: E731
    m = {"ova": PassiveAggressiveOneVersusAll.build_pa(L), "ova1": PassiveAggressiveOneVersusAll.build_pai(L, 1.0),
         "ova2": PassiveAggressiveOneVersusAll.build_paii(L, 1.0),
         "pb": PassiveAggressiveCostBased.build_pb(cost, L), "ml": PassiveAggressiveCostBased.build_ml(cost, L)}[method]
    train = _multi_data(300, F, L, 1)
    out = transform_multiclass(None, input_source=[Left(x) for x in train], worker_parallelism=2, ps_parallelism=2,
                               passive_aggressive_method=m, pull_limit=200, label_count=L, feature_count=F,
                               range_partitioning=False)
    W = np.zeros((F, L))
    for fid, vec in right_values(out):
        W[fid] = vec
    acc = multi_accuracy(W, _multi_data(100, F, L, 2), m)
    assert acc >= 80, acc


def test_cost_based_delta_not_accumulated():
    """each feature's delta is independent (the reference's builder leaks)."""
    m = PassiveAggressiveCostBased.build_pb(lambda y, q: 1.0, 3)
    x = SparseVector([0, 1], [1.0, 2.0], 4)
    model = {0: np.array([0.0, 1.0, 0.0]), 1: np.array([0.0, 1.0, 0.0])}
    d = dict(m.delta(x, model, 0))
    t = (3.0 - 0.0 + 1.0) / (2 * 5.0)
    np.testing.assert_allclose(d[0], [t, -t, 0])
    np.testing.assert_allclose(d[1], [2 * t, -2 * t, 0])


def test_multiclass_long_id_outputs_ids():
    F, L = 10, 2
    m = PassiveAggressiveOneVersusAll.build_pa(L)
    model = [(i, np.array([1.0, 0.0]) if i < 5 else np.array([0.0, 1.0])) for i in range(F)]
    inp = [Right((7, SparseVector([1], [1.0], F))), Right((8, SparseVector([9], [1.0], F)))]
    out = transform_multiclass_with_long_id(model, input_source=inp, worker_parallelism=1, ps_parallelism=2,
                                            passive_aggressive_method=m, pull_limit=10, label_count=L,
                                            feature_count=F, range_partitioning=True)
    assert sorted(left_values(out)) == [(7, 0), (8, 1)]


def _dict_data(n, F, seed, multi=False, L=3):
    rng = np.random.default_rng(seed)
    w = np.random.default_rng(99).normal(size=(F, L if multi else 1))
    out = []
    for _ in range(n):
        idx = rng.choice(F, size=6, replace=False)
        vals = rng.normal(size=6)
        x = {int(i): float(v) for i, v in zip(idx, vals)}
        s = vals @ w[idx]
        out.append((x, int(np.argmax(s)) if multi else (1 if s[0] > 0 else -1)))
    return out


@pytest.mark.parametrize("paf_type", [0, 1, 2])
def test_offline_binary_app(paf_type):
    from flink_parameter_server_1_amd.models.pa.offline import pa_binary_classification_offline

    train = _dict_data(400, 30, 1)
    test = _dict_data(100, 30, 2)
    out = pa_binary_classification_offline(train, [x for x, _ in test], worker_parallelism=2, ps_parallelism=2,
                                           iterations=5, paf_type=paf_type, paf_const=1, pull_limit=100, seed=0)
    preds = {tuple(sorted(v.items())): lab for v, lab in left_values(out)}
    acc = np.mean([preds[tuple(sorted(x.items()))] == y for x, y in test])
    assert len(preds) == len(test) and acc >= 0.8, acc


def test_offline_multiclass_app():
    from flink_parameter_server_1_amd.models.pa.offline import pa_multi_classification_offline

    train = _dict_data(600, 30, 1, multi=True)
    test = _dict_data(100, 30, 2, multi=True)
    out = pa_multi_classification_offline(train, [x for x, _ in test], label_count=3, worker_parallelism=2,
                                          ps_parallelism=3, iterations=5, paf_type=1, paf_const=1.0,
                                          pull_limit=100, seed=0)
    preds = {tuple(sorted(v.items())): lab for v, lab in left_values(out)}
    acc = np.mean([preds[tuple(sorted(x.items()))] == y for x, y in test])
    assert acc >= 0.7, acc


def test_filter_paii_is_float_division():
    from flink_parameter_server_1_amd.models.pa.offline import PassiveAggressiveFilter

    f = PassiveAggressiveFilter.build_pafii(2)
    d = f.delta({1: 1.0}, {1: 0.0}, 1)
    assert d[1] == pytest.approx(1.0 / (1.0 + 0.25))  # reference: 1/(2*2) == 0 in Int
