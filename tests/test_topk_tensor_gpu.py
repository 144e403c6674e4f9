"""Top-K tensor apps on the MI355X: MFMA scoring + LEMP masks + topk_merge_cand merge
equal the CPU reference paths."""
import numpy as np
import pytest
import torch

from flink_parameter_server_1_amd.models.mf.pruning import COORD, INCR, LI

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("strategy", [None, COORD(), INCR(4), LI(4, 1.2)])
def test_pruned_lemp_gpu_exact(strategy):
    from flink_parameter_server_1_amd.models.mf.topk_tensor import PrunedLempTopK

    g = torch.Generator().manual_seed(1)
    N, D, B, k = 40_000, 64, 128, 100
    X = (torch.randn(N, D, generator=g) * torch.rand(N, 1, generator=g)).to(DEV)
    Q = torch.randn(B, D, generator=g).to(DEV)
    ids = (torch.arange(N) * 3 + 1).to(DEV)
    idx = PrunedLempTopK(ids, X, bucket_size=4096, strategy=strategy)
    s, i = idx.query(Q, k)
    ts, tj = torch.topk(Q @ X.t(), k, dim=1)
    torch.testing.assert_close(s, ts, rtol=1e-4, atol=1e-4)
    assert (i == ids[tj]).float().mean() > 0.999  # fp32 ties aside


def test_merge_partials_gpu_matches_cpu():
    from flink_parameter_server_1_amd.models.mf.topk_tensor import merge_partials

    g = torch.Generator().manual_seed(2)
    B, m, K = 300, 600, 100
    s = torch.randn(B, m, generator=g)
    i = torch.randint(0, 10**6, (B, m), generator=g)
    exc = torch.rand(B, m, generator=g) < 0.2
    s[:, :5] = float("-inf")
    cs, ci = merge_partials(s, i, K, exc)
    gs, gi = merge_partials(s.to(DEV), i.to(DEV), K, exc.to(DEV))
    torch.testing.assert_close(gs.cpu(), cs)
    assert torch.equal(gi.cpu(), ci)


def test_topk_generator_tensor_gpu_matches_per_record():
    from flink_parameter_server_1_amd.core.messages import Left, Right
    from flink_parameter_server_1_amd.models.mf.apps import ps_top_k_generator
    from flink_parameter_server_1_amd.models.mf.core import Rating
    from flink_parameter_server_1_amd.models.mf.topk_tensor import as_reference_records, ps_top_k_generator_tensor
    from flink_parameter_server_1_amd.parallel.comm import Comm

    rng = np.random.default_rng(0)
    users, items, D = 40, 500, 16
    U = rng.normal(size=(users, D))
    V = rng.normal(size=(items, D)) * rng.random((items, 1))
    model = [Left((u, (float(np.linalg.norm(U[u])), U[u]))) for u in range(users)]
    model += [Right((i, (float(np.linalg.norm(V[i])), V[i]))) for i in range(items)]
    ratings = [Rating(int(rng.integers(0, users)), int(rng.integers(0, items)), 1.0, t) for t in range(64)]
    ref = ps_top_k_generator(ratings, model, num_factors=D, user_memory=8, K=20, worker_k=20, bucket_size=64,
                             pruning_algorithm=COORD(), worker_parallelism=1, ps_parallelism=1)
    ps_model = [(u, list(U[u]) + [float(np.linalg.norm(U[u]))]) for u in range(users)]
    w_model = [(i, list(V[i]) + [float(np.linalg.norm(V[i]))]) for i in range(items)]
    q = [(torch.tensor([r.user for r in ratings[s:s + 8]], device=DEV),
          torch.tensor([r.item for r in ratings[s:s + 8]], device=DEV),
          torch.tensor([r.timestamp for r in ratings[s:s + 8]], device=DEV)) for s in range(0, 64, 8)]
    out = ps_top_k_generator_tensor(q, ps_model, w_model, users, D, user_memory=8, K=20, worker_k=20,
                                    bucket_size=128, pruning_algorithm=COORD(), comm=Comm(device=DEV))
    got = as_reference_records(out)
    ref_by_ts = {ts: lst for (_, ts, lst) in ref}
    assert len(got) == 64
    for (u, it, ts, lst) in got:
        assert [x[1] for x in lst] == [x[1] for x in ref_by_ts[ts]]
