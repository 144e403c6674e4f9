"""LEMP top-K on the tensor path: MFMA scoring kernel, bucket early-exit, scatter-gather merge."""
import pytest
import torch

from dist_utils import run_ranks
from flink_parameter_server_1_amd import ops
from flink_parameter_server_1_amd.models.mf.topk_fast import DistributedTopK, LempTopK, merge_top_k


def _brute(Q, X, ids, k):
    s, j = torch.topk(Q @ X.T, k, dim=1)
    return s, ids[j]


def test_lemp_topk_exact_and_prunes():
    g = torch.Generator().manual_seed(0)
    X = torch.randn(5000, 16, generator=g) * torch.rand(5000, 1, generator=g) ** 4 * 3  # wide length spread
    ids = torch.arange(5000) * 3 + 1
    Q = torch.randn(40, 16, generator=g)
    lemp = LempTopK(ids, X, bucket_size=256)
    s, i = lemp.query(Q, 10)
    bs, bi = _brute(Q, X, ids, 10)
    torch.testing.assert_close(s, bs)
    assert torch.equal(i, bi)
    assert lemp.buckets_scanned < 5000 // 256 + 1  # the length bound skipped buckets


def test_merge_top_k_excludes_seen():
    s = torch.tensor([[0.9, 0.8, 0.7, 0.1]])
    i = torch.tensor([[5, 6, 7, 8]])
    ts, ti = merge_top_k(s, i, 2, exclude_ids=torch.tensor([[6, -1]]))
    assert ti.tolist() == [[5, 7]]


def _dist_topk(rank, world):
    g = torch.Generator().manual_seed(1)
    X = torch.randn(3000, 8, generator=g)
    Q = torch.randn(16, 8, generator=g)
    ids = torch.arange(3000)
    mine = ids % world == rank
    t = DistributedTopK(ids[mine], X[mine], bucket_size=128)
    ex = torch.full((16, 1), -1, dtype=torch.long)
    s, i = t.query(Q, 5, worker_k=5, exclude_ids=ex)
    bs, bi = _brute(Q, X, ids, 5)
    return torch.equal(i, bi) and torch.allclose(s, bs)


def test_distributed_topk_gloo():
    assert all(run_ranks(_dist_topk, 3))


@pytest.mark.gpu
@pytest.mark.parametrize("B,N,D", [(1, 1, 1), (64, 64, 32), (100, 1000, 64), (37, 5003, 100), (300, 70000, 10)])
def test_score_gemm_matches_matmul(B, N, D):
    g = torch.Generator().manual_seed(B + N)
    Q = torch.randn(B, D, generator=g)
    X = torch.randn(N, D, generator=g) + torch.arange(D)[None, :] * 0.01  # asymmetric operand
    S = ops.score_gemm(Q.cuda(), X.cuda()).cpu()
    torch.testing.assert_close(S, Q @ X.T, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_score_gemm_into_strided_slice():
    Q = torch.randn(50, 64, device="cuda")
    X = torch.randn(300, 64, device="cuda")
    buf = torch.full((50, 512), 7.0, device="cuda")
    ops.score_gemm(Q, X, buf[:, :300])
    torch.testing.assert_close(buf[:, :300], Q @ X.T, rtol=1e-5, atol=1e-4)
    assert bool((buf[:, 300:] == 7.0).all())


@pytest.mark.gpu
def test_lemp_topk_gpu_exact():
    g = torch.Generator().manual_seed(3)
    X = (torch.randn(200000, 64, generator=g) * torch.rand(200000, 1, generator=g) ** 3).cuda()
    ids = torch.arange(200000, device="cuda")
    Q = torch.randn(256, 64, generator=g).cuda()
    s, i = LempTopK(ids, X, bucket_size=16384).query(Q, 100)
    bs, bi = torch.topk(Q @ X.T, 100, dim=1)
    torch.testing.assert_close(s, bs, rtol=1e-5, atol=1e-4)
    assert float((i == bi).float().mean()) > 0.999  # ties may reorder


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4096, 1])
def test_lemp_topk_fused_equals_unfused(seed):
    """Fused scoring + filter (``ops.score_filter``) == the materialised-score scan; seed 1
    leaves the k-th best at ~-inf, so the fused segments overflow and rescan unfused."""
    g = torch.Generator().manual_seed(4)
    X = (torch.randn(100000, 64, generator=g) * torch.rand(100000, 1, generator=g) ** 2).cuda()
    ids = torch.arange(100000, device="cuda") * 3 + 1
    Q = torch.randn(300, 64, generator=g).cuda()
    fused = LempTopK(ids, X, bucket_size=16384)
    fused.seed_items = seed
    fused.geometric = seed != 1  # seed 1 + one 16383-item segment: the filter overflows
    s, i = fused.query(Q, 100)
    plain = LempTopK(ids, X, bucket_size=16384)
    plain.fused = False
    s0, i0 = plain.query(Q, 100)
    torch.testing.assert_close(s, s0, rtol=0, atol=0)
    assert float((i == i0).float().mean()) > 0.999
    assert (fused.overflows > 0) == (seed == 1)
    bs, _ = torch.topk(Q @ X.T, 100, dim=1)
    torch.testing.assert_close(s, bs, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_score_filter_counts_and_candidates():
    """Every score strictly above the row's k-th best is listed, with its item id."""
    torch.manual_seed(0)
    B, n, D, k = 130, 3000, 64, 10
    Q, X = torch.randn(B, D, device="cuda"), torch.randn(n, D, device="cuda")
    ids = torch.arange(n, device="cuda") + 100
    best_s = torch.sort(torch.randn(B, k, device="cuda") * 3 + 6, dim=1, descending=True)[0]
    cap = 512
    ck = torch.empty((B, cap), dtype=torch.int32, device="cuda")
    ci = torch.empty((B, cap), dtype=torch.long, device="cuda")
    cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    ops.score_filter(Q, X, ids, best_s, ck, ci, cnt)
    S = (Q.double() @ X.double().T).float().cpu()
    thr = best_s[:, -1].cpu()
    for b in range(B):
        want = set((torch.nonzero(S[b] > thr[b]).flatten() + 100).tolist())
        c = int(cnt[b])
        got = set(ci[b, :min(c, cap)].cpu().tolist())
        # scores within float rounding of the threshold may fall either way
        near = set((torch.nonzero((S[b] - thr[b]).abs() < 1e-4).flatten() + 100).tolist())
        assert got - near == want - near or c > cap


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 10, 100, 256])
@pytest.mark.parametrize("n", [100, 5000, 65536])
def test_topk_merge_kernel_exact(k, n):
    """Running-top-k merge kernel == torch.topk over [best, S] (two rounds: -inf start, then merge)."""
    torch.manual_seed(k + n)
    B = 64
    best_s = torch.full((B, k), float("-inf"), device="cuda")
    best_i = torch.full((B, k), -1, dtype=torch.long, device="cuda")
    ref_s, ref_i = best_s.cpu().clone(), best_i.cpu().clone()
    for rnd in range(2):
        S = torch.randn(B, n, device="cuda")
        if rnd == 1:
            S[:, : n // 3] += 2.0  # many new candidates above the running k-th best
        ids = torch.arange(n, device="cuda") + rnd * n
        ops.topk_merge(S, ids, best_s, best_i)
        cs = torch.cat([ref_s, S.cpu()], 1)
        ci = torch.cat([ref_i, ids.cpu().expand(B, n)], 1)
        kk = min(k, cs.shape[1])
        ts, tj = torch.topk(cs, kk, dim=1)
        ref_s[:, :kk], ref_i[:, :kk] = ts, torch.gather(ci, 1, tj)
        torch.testing.assert_close(best_s.cpu()[:, :kk], ref_s[:, :kk])
        # ids equal wherever the score is not tied with a neighbour (x + 2.0 rounds: ties happen)
        rs = ref_s[:, :kk]
        tie = torch.zeros_like(rs, dtype=torch.bool)
        tie[:, 1:] |= rs[:, 1:] == rs[:, :-1]
        tie[:, :-1] |= rs[:, :-1] == rs[:, 1:]
        same = (best_i.cpu()[:, :kk] == ref_i[:, :kk]) | tie
        assert bool(same.all())


def _updated_index(dev):
    g = torch.Generator().manual_seed(11)
    X = torch.randn(6000, 16, generator=g) * torch.rand(6000, 1, generator=g) ** 3
    ids = torch.arange(6000) * 2
    lemp = LempTopK(ids.to(dev), X.to(dev), bucket_size=512)
    # rewrite some rows in place (some get much longer: the length order breaks)
    rows = torch.randperm(6000, generator=g)[:300]
    newv = torch.randn(300, 16, generator=g) * 2
    X[rows] = newv
    pos = torch.empty(6000, dtype=torch.long)
    pos[lemp.order.cpu()] = torch.arange(6000)
    lemp.update_rows(pos[rows].to(dev), newv.to(dev))
    return lemp, X, ids


def test_lemp_topk_incremental_update_stays_exact():
    lemp, X, ids = _updated_index("cpu")
    Q = torch.randn(30, 16, generator=torch.Generator().manual_seed(12))
    s, i = lemp.query(Q, 10)
    bs, bi = _brute(Q, X, ids, 10)
    torch.testing.assert_close(s, bs)
    assert torch.equal(i, bi)


@pytest.mark.gpu
def test_lemp_topk_incremental_update_stays_exact_gpu():
    lemp, X, ids = _updated_index("cuda")
    lemp.seed_items = 256
    Q = torch.randn(200, 16, generator=torch.Generator().manual_seed(12))
    s, i = lemp.query(Q.cuda(), 10)
    bs, bi = _brute(Q, X, ids, 10)
    torch.testing.assert_close(s.cpu(), bs, rtol=1e-5, atol=1e-5)
    assert float((i.cpu() == bi).float().mean()) > 0.999


@pytest.mark.gpu
@pytest.mark.parametrize("D", [64, 33, 8])
@pytest.mark.parametrize("with_len", [False, True])
def test_score_filter_lemp_counts_and_candidates(with_len, D):
    """Fused scorer: every score strictly above the row's k-th best is listed;
    with lengths, skipped tiles hold no such score (the bound is exact)."""
    torch.manual_seed(1)
    B, n, k = 300, 5000, 10
    Q = torch.randn(B, D, device="cuda")
    X = torch.randn(n, D, device="cuda") * (torch.rand(n, 1, device="cuda") ** 4)  # many short items
    ids = torch.arange(n, device="cuda") + 7
    best_s = torch.sort(torch.randn(B, k, device="cuda") * 3 + D / 8, dim=1, descending=True)[0]
    best_s[:5] = float("-inf")  # rows still filling: everything passes
    cap = 2048
    ck = torch.empty((B, cap), dtype=torch.int32, device="cuda")
    ci = torch.empty((B, cap), dtype=torch.long, device="cuda")
    cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    ql = torch.linalg.vector_norm(Q, dim=1) if with_len else None
    xl = torch.linalg.vector_norm(X, dim=1) if with_len else None
    ops.score_filter_lemp(Q, X, ids, best_s, ck, ci, cnt, ql, xl)
    S = (Q.double() @ X.double().T).float().cpu()
    thr = best_s[:, -1].cpu()
    for b in range(B):
        want = set((torch.nonzero(S[b] > thr[b]).flatten() + 7).tolist())
        c = int(cnt[b])
        got = set(ci[b, :min(c, cap)].cpu().tolist())
        near = set((torch.nonzero((S[b] - thr[b]).abs() < 1e-4).flatten() + 7).tolist())
        assert got - near == want - near or c > cap, b
    assert int(cnt[:5].min()) == n  # -inf rows: all pass (5000 > cap: overflow reported by count)


@pytest.mark.gpu
def test_lemp_topk_sync_free_equals_synced_scan():
    g = torch.Generator().manual_seed(5)
    X = (torch.randn(150000, 64, generator=g) * torch.rand(150000, 1, generator=g) ** 2).cuda()
    ids = torch.arange(150000, device="cuda")
    Q = torch.randn(500, 64, generator=g).cuda()
    a = LempTopK(ids, X, bucket_size=16384)
    b = LempTopK(ids, X, bucket_size=16384)
    b.sync_free = False
    sa, ia = a.query(Q, 75)
    sb, ib = b.query(Q, 75)
    torch.testing.assert_close(sa, sb, rtol=0, atol=0)
    assert float((ia == ib).float().mean()) > 0.999
    assert a.overflows == 0


@pytest.mark.gpu
@pytest.mark.parametrize("nc_max", [40, 256, 900])  # rank path, its edge, bitonic path
@pytest.mark.parametrize("k", [75, 200])  # <= 64 / > 128 running entries per lane of the wave kernel
def test_topk_merge_cand_exact(nc_max, k):
    """Candidate merge == a (key desc, id asc) sort of running list + candidates, ties included."""
    from flink_parameter_server_1_amd.models.mf.topk_tensor import _fkey

    torch.manual_seed(nc_max + k)
    B, cap = 96, 1024
    best_s = torch.sort(torch.round(torch.randn(B, k) * 4) / 4, dim=1, descending=True)[0]
    best_s[:8, 40:] = float("-inf")  # rows still filling
    best_i = torch.randint(0, 10**6, (B, k))
    best_i[:8, 40:] = -1

    def ukey(x):  # the kernels' order-preserving key as a non-negative int64 (-0.0 < +0.0)
        return _fkey(x).to(torch.int64) & 0xFFFFFFFF

    # a running list sorted by (key desc, id asc), as the kernels keep it
    o = torch.argsort(best_i, dim=1, stable=True)
    best_s, best_i = torch.gather(best_s, 1, o), torch.gather(best_i, 1, o)
    o = torch.argsort(-ukey(best_s), dim=1, stable=True)
    best_s, best_i = torch.gather(best_s, 1, o), torch.gather(best_i, 1, o)
    cnt = torch.randint(0, nc_max + 1, (B,), dtype=torch.int32)
    cs = torch.round(torch.randn(B, cap) * 4) / 4  # coarse values: many ties
    ci = torch.randint(10**6, 2 * 10**6, (B, cap))
    ck = _fkey(cs)
    got_s, got_i = best_s.clone().cuda(), best_i.clone().cuda()
    ops.topk_merge_cand(ck.cuda(), ci.cuda(), cnt.cuda(), got_s, got_i)
    for b in range(B):
        n = int(cnt[b])
        s = torch.cat([best_s[b], cs[b, :n]])
        i = torch.cat([best_i[b], ci[b, :n]])
        o = torch.argsort(i, stable=True)
        s, i = s[o], i[o]
        o = torch.argsort(-ukey(s), stable=True)
        assert torch.equal(got_s[b].cpu(), s[o][:k]), b
        assert torch.equal(got_i[b].cpu(), i[o][:k]), b


@pytest.mark.gpu
@pytest.mark.parametrize("k,n", [(75, 4096), (100, 65536), (10, 300)])
def test_topk_merge_kernel_exact_with_ties(k, n):
    """Coarse scores (many ties at the k-th value): the radix threshold ends on the exact
    k-th key, so the kernel keeps the first k of a (key desc, id asc) order -- the seed
    segment of the LEMP scan merges 4096 x 4096 scores this way."""
    from flink_parameter_server_1_amd.models.mf.topk_tensor import _fkey

    g = torch.Generator().manual_seed(k + n)
    B = 48
    S = torch.round(torch.randn(B, n, generator=g) * 4) / 4
    ids = torch.randperm(10 * n, generator=g)[:n]
    best_s = torch.full((B, k), float("-inf"), device="cuda")
    best_i = torch.full((B, k), -1, dtype=torch.long, device="cuda")
    ops.topk_merge(S.cuda(), ids.cuda(), best_s, best_i)
    key = _fkey(S).to(torch.int64) & 0xFFFFFFFF
    for b in range(B):
        o = torch.argsort(ids, stable=True)
        kb, ib, sb = key[b][o], ids[o], S[b][o]
        o2 = torch.argsort(-kb, stable=True)[:k]
        assert torch.equal(best_s[b].cpu(), sb[o2]), b
        assert torch.equal(best_i[b].cpu(), ib[o2]), b
