"""Native per-record online-MF engine (csrc/host/record_engine.cpp) vs the Python
per-record engine with the same (hash) init: same protocol, same schedule, same
folded model."""
import numpy as np
import pytest

from flink_parameter_server_1_amd.core.messages import Left, Right
from flink_parameter_server_1_amd.models.mf.apps import ps_online_mf
from flink_parameter_server_1_amd.models.mf.core import FactorIsNotANumberException, Rating
from flink_parameter_server_1_amd.utils import native_host

pytestmark = pytest.mark.skipif(not native_host.available(), reason="host library not built")


def _fold(out):
    U, V = {}, {}
    for e in out:  # last-writer-wins fold of the output stream
        if isinstance(e, Left):
            U[e.value[0]] = np.asarray(e.value[1])
        elif isinstance(e, Right):
            V[e.value[0]] = np.asarray(e.value[1])
    return U, V


@pytest.mark.parametrize("W,P,limit,lam", [(1, 1, 1600, 0.0), (3, 2, 7, 0.0), (2, 3, 1600, 0.05), (4, 4, 3, 0.0)])
def test_native_equals_python_record_engine(W, P, limit, lam):
    from flink_parameter_server_1_amd.models.mf.native import ps_online_mf_native

    rng = np.random.default_rng(W * 10 + P)
    n = 3000
    u, i, r = rng.integers(0, 60, n), rng.integers(-20, 40, n), rng.random(n)  # negative ids: |id| % P
    kw = dict(num_factors=8, range_min=0.0, range_max=0.3, learning_rate=0.05, lam=lam, pull_limit=limit,
              worker_parallelism=W, ps_parallelism=P, seed=7)
    res = ps_online_mf_native(u, i, r, **kw)
    U, V = _fold(ps_online_mf([Rating(int(a), int(b), float(c), t) for t, (a, b, c) in enumerate(zip(u, i, r))],
                              init="hash", **kw))
    nu, nv = res.users(), res.items()
    assert set(U) == set(nu) and set(V) == set(nv)
    for k in U:
        np.testing.assert_allclose(nu[k], U[k], rtol=0, atol=1e-12)
    for k in V:
        np.testing.assert_allclose(nv[k], V[k], rtol=0, atol=1e-12)
    assert res.stats["pulls"] == res.stats["pushes"] == res.stats["answers"] == n


def test_native_negative_sampling_and_training():
    from flink_parameter_server_1_amd.models.mf.native import ps_online_mf_native

    rng = np.random.default_rng(1)
    users, items, rank, n = 200, 150, 4, 40000
    Ut, It = rng.random((users, rank)) / 2, rng.random((items, rank)) / 2
    u, i = rng.integers(0, users, n), rng.integers(0, items, n)
    r = (Ut[u] * It[i]).sum(1)
    res = ps_online_mf_native(u, i, r, num_factors=rank, range_min=0.0, range_max=0.3, learning_rate=0.05,
                              worker_parallelism=2, ps_parallelism=2)
    U, V = res.users(), res.items()
    err = np.sqrt(np.mean([(r[k] - U[u[k]] @ V[i[k]]) ** 2 for k in range(n)]))
    assert err < 0.1
    neg = ps_online_mf_native(u[:2000], i[:2000], r[:2000], num_factors=rank, negative_sample_rate=2,
                              user_memory=8, worker_parallelism=2, ps_parallelism=2)
    # every rating after the first few known items draws 2 negatives, each a pull + push
    assert neg.stats["negatives"] > 3000
    assert neg.stats["pulls"] == neg.stats["pushes"] == 2000 + neg.stats["negatives"]


def test_native_nan_raises():
    from flink_parameter_server_1_amd.models.mf.native import ps_online_mf_native

    with pytest.raises(FactorIsNotANumberException):
        ps_online_mf_native(np.array([1, 1]), np.array([2, 2]), np.array([np.nan, 1.0]), num_factors=4)
