"""Word2vec SGNS + negative sampling: CPU reference semantics, GPU kernels vs reference, gloo distributed."""
import numpy as np
import pytest
import torch

from dist_utils import run_ranks
from flink_parameter_server_1_amd import ops
from flink_parameter_server_1_amd.ops import reference as R


def test_alias_table_distribution():
    w = np.array([5.0, 1.0, 3.0, 1.0])
    prob, alias = ops.build_alias_table(w)
    s = ops.sample_alias(prob, alias, 200_000, seed=3)
    freq = torch.bincount(s.long(), minlength=4).double() / s.numel()
    np.testing.assert_allclose(freq.numpy(), w / w.sum(), atol=0.01)


def test_uniform_reject_avoids_positive_and_ring():
    pos = torch.tensor([0, 1, 2, 3], dtype=torch.int32)
    user = torch.tensor([0, 1, 0, 1], dtype=torch.int32)
    ring = torch.tensor([[4, 5], [6, -1]], dtype=torch.int32).flatten()
    out = ops.sample_uniform_reject(4, 50, 8, pos, user, ring, 2, seed=1).view(4, 50)
    for b in range(4):
        banned = {int(pos[b])} | ({4, 5} if user[b] == 0 else {6})
        assert not (set(out[b].tolist()) & banned)


def test_sgns_cpu_learns_cooccurrence():
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus

    cfg = SGNSConfig(vocab_size=2000, dim=16, window=3, learning_rate=0.025)
    m = DistributedSGNS(cfg)
    toks = synthetic_corpus(40000, 2000, n_topics=10, seed=1)
    c, o = skipgram_pairs(toks, 3, torch.Generator().manual_seed(0))
    first = m.step(c[:2048], o[:2048], with_loss=True)
    for s in range(0, c.numel() - 1024, 1024):
        m.step(c[s:s + 1024], o[s:s + 1024])
    last = m.step(c[:2048], o[:2048], with_loss=True)
    assert last < 0.8 * first, (first, last)


def _dist_sgns(rank, world):
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus

    m = DistributedSGNS(SGNSConfig(vocab_size=2000, dim=8, window=2, learning_rate=0.025))
    toks = synthetic_corpus(12000, 2000, n_topics=6, seed=rank)
    c, o = skipgram_pairs(toks, 2, torch.Generator().manual_seed(rank))
    first = m.step(c[:1024], o[:1024], with_loss=True)
    for s in range(60):  # every rank runs the same number of (collective) steps
        a = (s * 512) % (c.numel() - 512)
        m.step(c[a:a + 512], o[a:a + 512])
    return first, m.step(c[:1024], o[:1024], with_loss=True)


def test_sgns_distributed_gloo():
    res = run_ranks(_dist_sgns, 2)
    for first, last in res:
        assert last < first


# ----------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("D", [16, 64, 100, 300])
@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("runs", [False, True])
@pytest.mark.parametrize("neg_k,group", [(16, 1), (16, 2), (16, 4), (32, 1)])
def test_sgns_kernel_matches_reference(D, wire, runs, neg_k, group):
    torch.manual_seed(D)
    # groups: a partial last group (200 = 1.5 groups of 4 x 32 + 8)
    Uin, Uout, P = 300, 400, 200
    rows_in = (torch.randn(Uin, D) * 0.3).to(wire)
    rows_out = (torch.randn(Uout, D) * 0.3).to(wire)
    pos_c = torch.randint(0, Uin, (P,), dtype=torch.int32)
    if runs:  # center-major order: runs of equal centers (summed in LDS before the atomics)
        pos_c = torch.sort(torch.randint(0, 40, (P,), dtype=torch.int32)).values
    pos_o = torch.randint(0, Uout, (P,), dtype=torch.int32)
    pos_neg = torch.randint(0, Uout, (((P + 32 * group - 1) // (32 * group)) * neg_k,), dtype=torch.int32)
    d_in_r, d_out_r = torch.zeros(Uin, D), torch.zeros(Uout, D)
    loss_r = R.sgns_step(rows_in, rows_out, pos_c, pos_o, pos_neg, 0.05, 5 / neg_k, d_in_r, d_out_r, neg_k, group)
    dev = "cuda"
    d_in, d_out = torch.zeros(Uin, D, device=dev), torch.zeros(Uout, D, device=dev)
    loss = ops.sgns_step(rows_in.to(dev), rows_out.to(dev), pos_c.to(dev), pos_o.to(dev), pos_neg.to(dev), 0.05,
                         5 / neg_k, d_in, d_out, with_loss=True, neg_k=neg_k, neg_group=group)
    torch.testing.assert_close(d_in.cpu(), d_in_r, rtol=1e-4, atol=2e-6)
    torch.testing.assert_close(d_out.cpu(), d_out_r, rtol=1e-4, atol=2e-6)
    assert abs(float(loss) - loss_r) / loss_r < 1e-4


@pytest.mark.gpu
def test_sampling_kernels_match_reference():
    prob, alias = ops.build_alias_table(np.arange(1, 101, dtype=np.float64))
    a = ops.sample_alias(prob.cuda(), alias.cuda(), 10000, seed=5, counter=7).cpu()
    b = R.sample_alias(prob, alias, 10000, 5, 7)
    assert torch.equal(a, b)
    pos = torch.randint(0, 50, (300,), dtype=torch.int32)
    user = torch.randint(0, 10, (300,), dtype=torch.int32)
    ring = torch.randint(-1, 50, (10 * 4,), dtype=torch.int32)
    g = ops.sample_uniform_reject(300, 5, 50, pos.cuda(), user.cuda(), ring.cuda(), 4, seed=2, counter=9,
                                  device="cuda").cpu()
    c = R.sample_uniform_reject(300, 5, 50, pos, user, ring, 4, 2, 9)
    assert torch.equal(g, c)


@pytest.mark.gpu
def test_sgns_gpu_training_reduces_loss():
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus
    from flink_parameter_server_1_amd.parallel.comm import Comm

    m = DistributedSGNS(SGNSConfig(vocab_size=20000, dim=128, window=4, learning_rate=0.01),
                        comm=Comm(device=torch.device("cuda")))
    toks = synthetic_corpus(400000, 20000, n_topics=50, seed=1, device="cuda")
    c, o = skipgram_pairs(toks, 4)
    first = m.step(c[:8192], o[:8192], with_loss=True)
    for s in range(0, c.numel() - 8192, 8192):
        m.step(c[s:s + 8192], o[s:s + 8192])
    last = m.step(c[:8192], o[:8192], with_loss=True)
    assert last < 0.8 * first, (first, last)


def test_sgns_local_direct_matches_ps_path_on_one_rank():
    """W = 1 direct path (kernel updates the tables in place) trains like the PS
    path and its close-time dump covers the same touched rows."""
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus

    res = {}
    for direct in (True, False):
        torch.manual_seed(0)  # skipgram_pairs' reduced windows: the same pairs for both paths
        m = DistributedSGNS(SGNSConfig(vocab_size=2000, dim=32, learning_rate=0.005, local_direct=direct))
        assert m._direct == direct
        c, o = skipgram_pairs(synthetic_corpus(40000, 2000, seed=0), 5)
        l0 = m.step(c[:4096], o[:4096], with_loss=True)
        for i in range(30):
            s = (i * 4096) % (c.numel() - 4096)
            m.step(c[s:s + 4096], o[s:s + 4096])
        l1 = m.step(c[:4096], o[:4096], with_loss=True)
        ids, _ = m.embeddings()
        res[direct] = (l0, l1, set(ids.tolist()))
    assert res[True][1] < res[True][0] and res[False][1] < res[False][0]
    # (no closeness claim between the two: on the GPU the direct path is the sequential
    # in-place update -- it equals the sequential reference loop, see
    # test_sgns_direct_path_equals_sequential_reference -- while the PS path reads one
    # pulled snapshot per micro-batch; at 4096 pairs over 2000 words the sequential form
    # learns ~10x faster per step (3.91 vs 4.14 from 4.15), so the round-5 5 % bound held
    # only for lucky reduced-window draws)
    # both dumps cover every word that occurred; rows touched only as sampled negatives
    # may differ (the two paths draw their negatives from different streams)
    seen = set(c[:4096].tolist()) | set(o[:4096].tolist())
    assert seen <= res[True][2] and seen <= res[False][2]
    assert len(res[True][2] ^ res[False][2]) <= 0.01 * len(res[False][2])


# ----------------------------------------------------------- standard SGNS
def test_sgns_standard_loop_equals_batched_without_shared_rows():
    """No center runs, no row shared between pairs: the kernel's sequential order
    (reference.sgns_standard) and the CPU mini-batch form agree."""
    torch.manual_seed(0)
    P, k, D = 40, 5, 12
    rows_in, rows_out = torch.randn(P, D) * 0.3, torch.randn(P * (k + 1), D) * 0.3
    pos_c = torch.arange(P, dtype=torch.int32)
    perm = torch.randperm(P * (k + 1)).to(torch.int32)
    pos_o, pos_neg = perm[:P], perm[P:]
    outs = []
    for fn in (R.sgns_standard, R.sgns_standard_batched):
        d_in, d_out = torch.zeros(P, D), torch.zeros(P * (k + 1), D)
        loss = fn(rows_in, rows_out, pos_c, pos_o, pos_neg, k, 0.05, d_in, d_out)
        outs.append((d_in, d_out, loss))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-7)
    assert abs(outs[0][2] - outs[1][2]) < 1e-6 * outs[1][2]


def test_sgns_standard_skips_negative_equal_to_context():
    rows_in, rows_out = torch.ones(1, 4), torch.ones(3, 4) * 0.1
    d_in, d_out = torch.zeros(1, 4), torch.zeros(3, 4)
    R.sgns_standard_batched(rows_in, rows_out, torch.tensor([0]), torch.tensor([1]), torch.tensor([1, 2]), 2, 0.1,
                            d_in, d_out)
    g_o = 0.1 * (1 - torch.sigmoid(torch.tensor(0.4)))
    torch.testing.assert_close(d_out[1], g_o * torch.ones(4))  # only the positive update on row 1


@pytest.mark.parametrize("mode", ["standard", "shared"])
def test_sgns_modes_learn_on_cpu(mode):
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus

    m = DistributedSGNS(SGNSConfig(vocab_size=2000, dim=16, window=3, learning_rate=0.025, mode=mode))
    toks = synthetic_corpus(40000, 2000, n_topics=10, seed=1)
    c, o = skipgram_pairs(toks, 3, torch.Generator().manual_seed(0))
    first = m.step(c[:2048], o[:2048], with_loss=True)
    for s in range(0, c.numel() - 1024, 1024):
        m.step(c[s:s + 1024], o[s:s + 1024])
    assert m.step(c[:2048], o[:2048], with_loss=True) < 0.8 * first


@pytest.mark.gpu
@pytest.mark.parametrize("D", [16, 64, 100, 300])
@pytest.mark.parametrize("runs", [False, True])
@pytest.mark.parametrize("k", [1, 5, 7])
@pytest.mark.parametrize("method", ["sorted", "atomic"])
def test_sgns_standard_kernel_matches_reference(D, runs, k, method):
    """PS-path form (rows read-only, separate delta buffers): the kernel equals the
    sequential reference, center runs included (float-atomic order aside)."""
    torch.manual_seed(D + k)
    Uin, Uout, P = 300, 400, 3000
    rows_in = torch.randn(Uin, D) * 0.3
    rows_out = torch.randn(Uout, D) * 0.3
    pos_c = torch.randint(0, Uin, (P,), dtype=torch.int32)
    if runs:  # center-major: runs of equal centers, sequential inside a wave's chunk
        pos_c = torch.sort(torch.randint(0, 60, (P,), dtype=torch.int32)).values
    pos_o = torch.randint(0, Uout, (P,), dtype=torch.int32)
    pos_neg = torch.randint(0, Uout, (P * k,), dtype=torch.int32)
    d_in_r, d_out_r = torch.zeros(Uin, D), torch.zeros(Uout, D)
    loss_r = R.sgns_standard(rows_in, rows_out, pos_c, pos_o, pos_neg, k, 0.05, d_in_r, d_out_r, method=method)
    dev = "cuda"
    d_in, d_out = torch.zeros(Uin, D, device=dev), torch.zeros(Uout, D, device=dev)
    loss = ops.sgns_standard(rows_in.to(dev), rows_out.to(dev), pos_c.to(dev), pos_o.to(dev), pos_neg.to(dev), k,
                             0.05, d_in, d_out, with_loss=True, method=method)
    torch.testing.assert_close(d_in.cpu(), d_in_r, rtol=1e-4, atol=5e-6)
    torch.testing.assert_close(d_out.cpu(), d_out_r, rtol=1e-4, atol=5e-6)
    assert abs(float(loss) - loss_r) / loss_r < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("D", [16, 64, 100, 300, 512])
@pytest.mark.parametrize("method", ["sorted", "atomic"])
def test_sgns_standard_bf16_rows_match_reference(D, method):
    """bf16 pulled rows (the PS path's bf16 wire) read by the kernels directly, as
    coordinate pairs widened in registers: the same deltas as the sequential reference
    on the widened rows (the per-lane summation order differs from the fp32 layout)."""
    torch.manual_seed(D + 1)
    k, Uin, Uout, P = 5, 300, 400, 3000
    rows_in = (torch.randn(Uin, D) * 0.3).bfloat16()
    rows_out = (torch.randn(Uout, D) * 0.3).bfloat16()
    pos_c = torch.sort(torch.randint(0, 60, (P,), dtype=torch.int32)).values
    pos_o = torch.randint(0, Uout, (P,), dtype=torch.int32)
    pos_neg = torch.randint(0, Uout, (P * k,), dtype=torch.int32)
    d_in_r, d_out_r = torch.zeros(Uin, D), torch.zeros(Uout, D)
    loss_r = R.sgns_standard(rows_in.float(), rows_out.float(), pos_c, pos_o, pos_neg, k, 0.05, d_in_r, d_out_r,
                             method=method)
    dev = "cuda"
    d_in, d_out = torch.zeros(Uin, D, device=dev), torch.zeros(Uout, D, device=dev)
    loss = ops.sgns_standard(rows_in.to(dev), rows_out.to(dev), pos_c.to(dev), pos_o.to(dev), pos_neg.to(dev), k,
                             0.05, d_in, d_out, with_loss=True, method=method)
    torch.testing.assert_close(d_in.cpu(), d_in_r, rtol=1e-4, atol=5e-6)
    torch.testing.assert_close(d_out.cpu(), d_out_r, rtol=1e-4, atol=5e-6)
    assert abs(float(loss) - loss_r) / loss_r < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("D", [64, 300])
@pytest.mark.parametrize("method", ["sorted", "atomic"])
def test_sgns_standard_bf16_push_output(D, method):
    """``d_out_bf16``: the output-row deltas leave the kernel in bf16 (the PS path's bf16
    push) with ``d_out`` as unzeroed scratch.  A very hot context row spans many of the
    rows kernel's 256-entry ranges (cut runs: zeroed, summed by atomics, narrowed after);
    every row equals bf16 of the reference delta (within the fp32 sums' rounding)."""
    torch.manual_seed(D + 7)
    k, Uin, Uout, P = 5, 300, 400, 3000
    rows_in = (torch.randn(Uin, D) * 0.3).bfloat16()
    rows_out = (torch.randn(Uout, D) * 0.3).bfloat16()
    pos_c = torch.sort(torch.randint(0, 60, (P,), dtype=torch.int32)).values
    pos_o = torch.where(torch.rand(P) < 0.4, 7, torch.randint(0, Uout, (P,))).to(torch.int32)  # row 7: 1200 entries
    pos_neg = torch.randint(0, Uout, (P * k,), dtype=torch.int32)
    d_in_r, d_out_r = torch.zeros(Uin, D), torch.zeros(Uout, D)
    R.sgns_standard(rows_in.float(), rows_out.float(), pos_c, pos_o, pos_neg, k, 0.05, d_in_r, d_out_r, method=method)
    dev = "cuda"
    d_in = torch.zeros(Uin, D, device=dev)
    d_out = torch.full((Uout, D), 123.0, device=dev)  # scratch: garbage on entry
    out_bf = torch.empty(Uout, D, dtype=torch.bfloat16, device=dev)
    ops.sgns_standard(rows_in.to(dev), rows_out.to(dev), pos_c.to(dev), pos_o.to(dev), pos_neg.to(dev), k, 0.05,
                      d_in, d_out, method=method, d_out_bf16=out_bf)
    torch.testing.assert_close(d_in.cpu(), d_in_r, rtol=1e-4, atol=5e-6)
    torch.testing.assert_close(out_bf.cpu().float(), d_out_r.bfloat16().float(), rtol=1.6e-2, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("D", [64, 300])
def test_sgns_standard_sorted_in_place_matches_reference(D):
    """Local path (d_in is rows_in, d_out is rows_out; a few very hot output rows
    shared by many waves): the sorted form equals its sequential reference -- the
    output rows take g * (center row after the pass's center updates).  Center runs
    are 8 pairs, aligned to the kernel's 16-pair waves, so no center row is shared
    between waves and the result is deterministic up to summation order."""
    torch.manual_seed(D)
    V, P, k = 5000, 16000, 5
    w_in = torch.randn(V, D) * 0.1
    w_out = torch.randn(V, D) * 0.1
    pos_c = torch.randperm(V)[:P // 8].to(torch.int32).repeat_interleave(8)
    pos_o = (torch.rand(P) ** 4 * V).to(torch.int32)  # Zipf-ish: a few very hot context rows
    pos_neg = torch.randint(0, V, (P * k,), dtype=torch.int32)
    d_in = torch.zeros_like(w_in)
    loss_r = R.sgns_standard(w_in, w_out, pos_c, pos_o, pos_neg, k, 0.05, d_in, torch.zeros_like(w_out))
    wi_post = w_in + d_in
    wo_post = w_out + _deferred_out(w_in, w_out, wi_post, pos_c, pos_o, pos_neg, k, 0.05)
    dev = "cuda"
    wi, wo = w_in.to(dev), w_out.to(dev)
    loss = ops.sgns_standard(wi, wo, pos_c.to(dev), pos_o.to(dev), pos_neg.to(dev), k, 0.05, wi, wo,
                             with_loss=True, method="sorted")
    torch.testing.assert_close(wi.cpu(), wi_post, rtol=1e-4, atol=5e-6)
    torch.testing.assert_close(wo.cpu(), wo_post, rtol=1e-4, atol=2e-5)
    assert abs(float(loss) - loss_r) / loss_r < 1e-4


def _deferred_out(rows_in, rows_out, h_rows, pos_c, pos_o, pos_neg, k, lr):
    """Output-row deltas of the sorted form: g from the sequential pass (runs of
    SGNS_STD_CHUNK pairs), times ``h_rows[center]``."""
    import math

    P, D = pos_c.numel(), rows_in.shape[1]
    out = torch.zeros(rows_out.shape[0], D, dtype=torch.float64)
    pc, po, pn = pos_c.tolist(), pos_o.tolist(), pos_neg.reshape(P, k).tolist()
    for s0 in range(0, P, R.SGNS_STD_CHUNK):
        cur, h = -1, None
        for p in range(s0, min(P, s0 + R.SGNS_STD_CHUNK)):
            if pc[p] != cur:
                cur, h = pc[p], rows_in[pc[p]].double().clone()
            dh = torch.zeros(D, dtype=torch.float64)
            for x, lab in [(po[p], 1.0)] + [(n, 0.0) for n in pn[p] if n != po[p]]:
                xv = rows_out[x].double()
                g = lr * (lab - 1.0 / (1.0 + math.exp(-float(h @ xv))))
                out[x] += g * h_rows[cur].double()
                dh += g * xv
            h = h + dh
    return out.float()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["standard", "shared"])
def test_sgns_gpu_modes_reduce_loss(mode):
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus
    from flink_parameter_server_1_amd.parallel.comm import Comm

    m = DistributedSGNS(SGNSConfig(vocab_size=20000, dim=300, window=4, learning_rate=0.01, mode=mode),
                        comm=Comm(device=torch.device("cuda")))
    toks = synthetic_corpus(400000, 20000, n_topics=50, seed=1, device="cuda")
    c, o = skipgram_pairs(toks, 4)
    first = m.step(c[:8192], o[:8192], with_loss=True)
    for s in range(0, c.numel() - 8192, 8192):
        m.step(c[s:s + 8192], o[s:s + 8192])
    assert m.step(c[:8192], o[:8192], with_loss=True) < 0.8 * first


# ----------------------------------------------------------- SGNS PS path: planning
def test_sgns_ps_plans_always_deduplicate_at_large_vocab_ratio():
    """The kernels find "negative == context" and center runs by comparing plan
    positions, so SGNS tables never get request plans -- even at a vocab / batch
    ratio far above TensorPS.REQUEST_PLAN_RATIO."""
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig

    V, P = 200_000, 256
    m = DistributedSGNS(SGNSConfig(vocab_size=V, dim=16, learning_rate=0.01, local_direct=False))
    assert V >= m.ps_in.REQUEST_PLAN_RATIO * P * (1 + m.cfg.negatives)
    assert m.ps_in.dedups(P) and m.ps_out.dedups(P * (1 + m.cfg.negatives))
    g = torch.Generator().manual_seed(0)
    c = torch.randint(0, 50, (P,), generator=g, dtype=torch.int32)  # repeated centers: runs must merge
    o = torch.randint(0, V, (P,), generator=g, dtype=torch.int32)
    for _ in range(3):
        m.step(c, o)
    m.flush()
    st = m.ps_in.stats
    assert st["unique"] <= 50 * st["steps"] < st["pulls"]


def test_sgns_ps_path_both_tables_share_one_plan_exchange():
    """Both tables are planned by one ``plan_begin_multi`` (one count exchange, one
    host copy) one micro-batch ahead: the pipelined steps equal the synchronous ones
    up to the staleness of one batch, and the last flush applies everything."""
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus
    from flink_parameter_server_1_amd.parallel.tensor_ps import TensorPS

    calls = []
    orig = TensorPS.plan_begin_multi

    def spy(pss, keys, flag=0, dedup=None):
        calls.append(len(pss))
        return orig(pss, keys, flag, dedup)

    TensorPS.plan_begin_multi = staticmethod(spy)
    try:
        m = DistributedSGNS(SGNSConfig(vocab_size=3000, dim=16, learning_rate=0.01, local_direct=False))
        c, o = skipgram_pairs(synthetic_corpus(20000, 3000, seed=2), 4)
        l0 = m.step(c[:2048], o[:2048], with_loss=True)
        for i in range(30):
            s = (i * 2048) % (c.numel() - 2048)
            m.step(c[s:s + 2048], o[s:s + 2048])
        assert m.pipe.in_flight + m.pipe.planned >= 1  # one batch still in the pipeline
        l1 = m.step(c[:2048], o[:2048], with_loss=True)  # drains first
    finally:
        TensorPS.plan_begin_multi = staticmethod(orig)
    assert calls and all(n == 2 for n in calls) and len(calls) == 32
    assert l1 < l0


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", [True, False])
def test_sgns_ps_path_steady_state_never_idles_the_device_on_counts(pipeline):
    """Pipelined: every plan_end finds later work enqueued behind its counts (zero
    device-idling host stalls); synchronous (pipeline=False): each step's counts are
    the newest work on the stream, so the host drains the device every step."""
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus
    from flink_parameter_server_1_amd.parallel.comm import Comm

    m = DistributedSGNS(SGNSConfig(vocab_size=100_000, dim=128, learning_rate=0.01, local_direct=False,
                                   pipeline=pipeline), comm=Comm(device=torch.device("cuda")))
    c, o = skipgram_pairs(synthetic_corpus(400_000, 100_000, seed=1, device="cuda"), 4)
    P = 1 << 16
    for i in range(4):  # warm-up
        m.step(c[i * P:(i + 1) * P], o[i * P:(i + 1) * P])
    m.flush()
    torch.cuda.synchronize()
    s0 = dict(m.ps_in.stats), dict(m.ps_out.stats)
    for i in range(20):
        s = ((i + 4) * P) % (c.numel() - P)
        m.step(c[s:s + P], o[s:s + P])
    # steady state only: the final flush plans nothing behind the last batch's counts
    stalls = [ps.stats["host_stalls"] - s["host_stalls"] for ps, s in zip((m.ps_in, m.ps_out), s0)]
    m.flush()
    torch.cuda.synchronize()
    if pipeline:
        assert stalls == [0, 0], stalls
    else:  # both tables' counts share one event: the first plan_end waits, the second finds it done
        assert stalls[0] >= 10 and stalls[1] == 0, stalls


def _sgns_ps_fused(device, fuse):
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus
    from flink_parameter_server_1_amd.parallel.comm import Comm

    m = DistributedSGNS(SGNSConfig(vocab_size=3000, dim=40, learning_rate=0.01, local_direct=False,
                                   fuse_local_push=fuse), comm=Comm(device=torch.device(device)))
    c, o = skipgram_pairs(synthetic_corpus(30000, 3000, seed=4, device=device), 4,
                          torch.Generator(device=device).manual_seed(1))
    for i in range(12):
        s = (i * 2048) % (c.numel() - 2048)
        m.step(c[s:s + 2048], o[s:s + 2048])
    m.flush()
    ids, w = m.embeddings()
    return ids.cpu(), w.cpu(), m.w_out.weight.cpu().clone(), dict(m.ps_in.stats)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_sgns_ps_path_fused_local_push_equals_pushed_deltas(device):
    """World 1: the kernel adding its pushes straight into the tables (write maps =
    the plans' rows) == delta buffers pushed and applied, reading the same pulled
    snapshots one batch stale (GPU: float atomics, summation order only)."""
    a = _sgns_ps_fused(device, True)
    b = _sgns_ps_fused(device, False)
    assert torch.equal(a[0], b[0])
    tol = dict(rtol=0, atol=0) if device == "cpu" else dict(rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(a[1], b[1], **tol)
    torch.testing.assert_close(a[2], b[2], **tol)
    assert a[3]["pushes"] == b[3]["pushes"] > 0


@pytest.mark.gpu
def test_sgns_direct_path_equals_sequential_reference():
    """The W = 1 direct path on the GPU (kernel updates the tables in place) trains like
    the sequential reference loop (``reference.sgns_standard``, sorted output-row form,
    in place) on the same pairs and negatives."""
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus

    torch.manual_seed(0)
    m = DistributedSGNS(SGNSConfig(vocab_size=2000, dim=32, learning_rate=0.005, local_direct=True))
    assert m._direct and m.w_in.weight.is_cuda
    c, o = skipgram_pairs(synthetic_corpus(40000, 2000, seed=0), 5)
    w_in, w_out = m.w_in.weight.cpu().clone(), m.w_out.weight.cpu().clone()
    counter = m.counter
    steps = [(0, True)] + [((i * 4096) % (c.numel() - 4096), False) for i in range(30)] + [(0, True)]
    got, ref = [], []
    for s, wl in steps:
        cc, oo = c[s:s + 4096], o[s:s + 4096]
        negs = ops.sample_alias(m.prob, m.alias, 4096 * 5, seed=m.cfg.seed, counter=counter).cpu().to(torch.int32)
        counter += 1
        d_out = torch.zeros_like(w_out)
        lr_ = R.sgns_standard(w_in, w_out, cc, oo, negs, 5, 0.005, w_in, d_out, method="sorted")
        w_out += d_out
        lg = m.step(cc.cuda(), oo.cuda(), with_loss=wl)
        if wl:
            got.append(lg)
            ref.append(lr_ / 4096)
    assert abs(got[0] - ref[0]) < 1e-4 * ref[0]
    assert abs(got[-1] - ref[-1]) < 0.01 * ref[-1], (got, ref)
