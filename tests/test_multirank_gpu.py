"""Multi-rank rehearsal on ONE GPU: 2-3 ranks share cuda:0 over gloo (host-staged
transport, parallel/comm.py), so the device code of the N > 1 paths -- tile partition
with side-stream prefetch, ring rotation, PS all-to-alls, locks -- runs on real
kernels.  RCCL itself is exercised only by the driver's 8-GPU run."""
import pytest
import torch

from dist_utils import run_ranks

pytestmark = pytest.mark.gpu


def _mf(rank, world, exchange):
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm(device=torch.device("cuda", 0))
    cfg = MFConfig(num_users=30000, num_items=4000, dim=64, learning_rate=0.05, range_min=0.0, range_max=0.2,
                   exchange=exchange)
    m = DistributedMF(cfg, comm)
    data = SyntheticRatings(30000, 4000, 1 << 19, rank, world, seed=9, truth_dim=8, device="cuda")
    before = m.rmse(*data.batch(0, 1 << 17))
    for s in range(20):
        m.step(*data.batch(s % 4, 1 << 17))
    after = m.rmse(*data.batch(0, 1 << 17))
    ids, _ = m.item_vectors(only_touched=True)
    rated = torch.unique(data.iid).cpu()
    return before, after, m.sgd_mode, ids.cpu(), rated


@pytest.mark.parametrize("world,exchange", [(2, "rotate"), (3, "rotate"), (2, "ps")])
def test_mf_multirank_on_one_gpu(world, exchange):
    res = run_ranks(_mf, world, exchange)
    before, after = res[0][0], res[0][1]
    assert after < 0.6 * before, (before, after)
    assert all(abs(r[1] - after) < 1e-9 for r in res)  # global RMSE
    if exchange == "rotate":
        assert res[0][2] == "tiled"
    # the close-time dump covers exactly the items some rank rated
    dumped = torch.sort(torch.cat([r[3] for r in res])).values
    rated = torch.unique(torch.cat([r[4] for r in res]))
    assert torch.equal(dumped, rated)


def _pair_locked(rank, world):
    from flink_parameter_server_1_amd.models.emb import DistributedPairEmbedding, PairEmbeddingConfig, synthetic_pairs
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.parallel.locked_ps import LockedTensorPS
    from flink_parameter_server_1_amd.parallel.table import ShardedTable

    comm = Comm(device=torch.device("cuda", 0))
    cfg = PairEmbeddingConfig(num_ids=300_000_000, dim=32, learning_rate=0.05, staleness=2, optimizer="adagrad")
    m = DistributedPairEmbedding(cfg, comm)
    batches = [synthetic_pairs(cfg.num_ids, 1 << 15, seed=rank + 1, step=s, device="cuda", zipf=3.0)
               for s in range(4)]
    before = m.mean_loss(*batches[0])
    for s in range(24):
        m.step(*batches[s % 4])
    after = m.mean_loss(*batches[0])
    # device locks: concurrent increments of shared counters are exact
    tab = ShardedTable(64, 1, comm.rank, comm.world, "hash", ("zeros",), device="cuda", track_touched=False)
    lps = LockedTensorPS(tab, comm)
    pending = torch.full((64,), 3, dtype=torch.int64)
    for _ in range(40):
        if comm.sum_over_ranks(float(pending.sum())) == 0:
            break
        keys = torch.nonzero(pending).flatten().to(torch.int32).cuda()
        pull = lps.acquire(keys)
        lps.release(pull, pull.rows.float() + 1.0, mode="set")
        pending[keys[pull.granted[pull.plan.pos.long()]].long().cpu()] -= 1
    _, vals = tab.dump(only_touched=False)
    return before, after, float(vals.sum()), lps.held()


def test_pair_embedding_and_locks_multirank_on_one_gpu():
    res = run_ranks(_pair_locked, 2)
    assert res[0][1] < res[0][0] - 0.1
    assert sum(r[2] for r in res) == 64 * 3 * 2  # every locked increment landed once
    assert all(r[3] == 0 for r in res)


def _w2v(rank, world):
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus
    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm(device=torch.device("cuda", 0))
    m = DistributedSGNS(SGNSConfig(vocab_size=20000, dim=128, window=4, learning_rate=0.01), comm=comm)
    assert m._pipelined
    toks = synthetic_corpus(200000, 20000, n_topics=50, seed=rank, device="cuda")
    c, o = skipgram_pairs(toks, 4)
    first = m.step(c[:8192], o[:8192], with_loss=True)
    for s in range(40):  # same number of collective steps on every rank
        a = (s * 8192) % (c.numel() - 8192)
        m.step(c[a:a + 8192], o[a:a + 8192])
    return first, m.step(c[:8192], o[:8192], with_loss=True)


def test_w2v_pipelined_multirank_on_one_gpu():
    res = run_ranks(_w2v, 2)
    for first, last in res:
        assert last < 0.97 * first, (first, last)  # learning (not a convergence test)


def _pa_plans(rank, world):
    """PA through the PS path with request plans (the routing kernel at W > 1) and with
    de-duplicating plans: the same model, on real kernels."""
    from flink_parameter_server_1_amd.models.pa.fast import DistributedPA, PAConfig, synthetic_sparse_batch
    from flink_parameter_server_1_amd.parallel.comm import Comm

    F = 1 << 26
    out = []
    for dedup in (True, False):
        m = DistributedPA(PAConfig(feature_count=F, kind="binary", local_direct=False),
                          Comm(device=torch.device("cuda", 0)))
        m.ps.dedup_mode = dedup
        for s in range(8):
            m.train_step(*synthetic_sparse_batch(2048, 32, F, seed=rank + 3, step=s % 4, device="cuda"))
        ids, w = m.dump()
        o = torch.argsort(ids)
        out.append((ids[o].cpu(), w[o].reshape(-1).cpu()))
    return out


def test_pa_request_plans_multirank_on_one_gpu():
    for (ia, wa), (ib, wb) in run_ranks(_pa_plans, 2):
        assert torch.equal(ia, ib)
        torch.testing.assert_close(wa, wb, rtol=2e-3, atol=1e-5)  # fp32 summation order (tests/test_pa_fast.py)
