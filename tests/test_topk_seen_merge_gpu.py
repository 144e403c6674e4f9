"""One-launch seen-aware merge (``ops.topk_seen_merge``, ``topk.hip`` ``seen_merge_kernel``)
against the round-by-round torch merge it replaces (``RoundPlan`` rounds +
``merge_partials`` + ``SeenStore.add``): identical top-K lists and identical ring
state, with users repeated inside the batch (also more often than the window) and
recommended items already in the users' windows."""
import pytest
import torch

from flink_parameter_server_1_amd import ops
from flink_parameter_server_1_amd.models.mf.topk_tensor import RoundPlan, SeenStore, merge_partials

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _reference(ss, ii, K, users, items, store):
    plan = RoundPlan(users)
    best_s = torch.empty((users.numel(), K), device=DEV)
    best_i = torch.empty((users.numel(), K), dtype=torch.long, device=DEV)
    for a, n in plan.rounds():
        sel = plan.order[a:a + n]
        exc = store.contains(users[sel], ii[sel])
        bs, bi = merge_partials(ss[sel], ii[sel], K, exc)
        best_s[sel], best_i[sel] = bs, bi
        store.add(users[sel], items[sel])
    return best_s, best_i


def _sort_rows(ss, ii):
    """Each row in the merge order (key desc, then id asc), invalid entries (-inf / id < 0)
    last as (-inf, -1): a single shard's sorted top-K list, the kernel's compaction path."""
    from flink_parameter_server_1_amd.models.mf.topk_tensor import _fkey

    bad = (ii < 0) | ~torch.isfinite(ss)
    ss = torch.where(bad, torch.full_like(ss, float("-inf")), ss)
    ii = torch.where(bad, torch.full_like(ii, -1), ii)
    key = _fkey(ss).to(torch.int64) & 0xFFFFFFFF
    key = torch.where(bad, torch.full_like(key, -1), key)
    o = torch.argsort(torch.where(bad, torch.full_like(ii, 2**62), ii), dim=1, stable=True)
    ss, ii, key = ss.gather(1, o), ii.gather(1, o), key.gather(1, o)
    o = torch.argsort(-key, dim=1, stable=True)
    return ss.gather(1, o).contiguous(), ii.gather(1, o).contiguous()


@pytest.mark.parametrize("sorted_rows", [False, True])
@pytest.mark.parametrize("m,K,memory", [(75, 100, 16), (600, 100, 16), (300, 50, 4), (64, 256, 256), (256, 100, 16)])
def test_seen_merge_equals_round_loop(m, K, memory, sorted_rows):
    g = torch.Generator(device=DEV).manual_seed(m + K)
    U, I, B = 500, 3000, 700
    ref_store = SeenStore(memory, DEV, num_users=U)
    new_store = SeenStore(memory, DEV, num_users=U)
    assert ref_store.ring is not None
    for step in range(3):
        users = torch.randint(0, U, (B,), device=DEV, generator=g)
        users[:40] = 7  # one user more often than its window
        users[40:45] = 11
        items = torch.randint(0, I, (B,), device=DEV, generator=g)
        ii = torch.randint(0, I, (B, m), device=DEV, generator=g)
        ii[:, ::9] = -1  # empty slots
        # recommend items the users rated in this batch / earlier batches
        ii[:, 1] = items.roll(1)
        ii[:, 2] = items
        ss = torch.randn(B, m, device=DEV, generator=g)
        ss[:, ::13] = float("-inf")
        ss[:, 5] = ss[:, 6]  # ties: smaller id first
        if sorted_rows:  # rows of m <= 256 take the kernel's sorted-input compaction
            ss, ii = _sort_rows(ss, ii)
        rs, ri = _reference(ss, ii, K, users, items, ref_store)
        plan = RoundPlan(users, fused=True)
        bs, bi = ops.topk_seen_merge(ss, ii, K, users, items, plan.rnd, plan.first, plan.nu, plan.by_user,
                                     new_store.ring, new_store.ring_cur)
        assert torch.equal(bs, rs), step
        assert torch.equal(bi, ri), step
        assert torch.equal(new_store.ring, ref_store.ring) and torch.equal(new_store.ring_cur, ref_store.ring_cur)


def _run_online(fused, batches, users, items, D, neg=0):
    from flink_parameter_server_1_amd.core.messages import Left
    from flink_parameter_server_1_amd.core.tensor_engine import TensorRuntime
    from flink_parameter_server_1_amd.models.mf.topk_tensor import OnlineMFTopKWorker
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogic

    w = OnlineMFTopKWorker(items, D, 0.05, K=20, worker_k=20, memory=8, negative_sample_rate=neg,
                           prefill_items=True, num_users=users, resort_every=1000, range_min=-0.3, range_max=0.3)
    w.fused = fused
    logic = DeviceSimplePSLogic(users, D, op="add_renorm", init=("uniform", -0.3, 0.3))
    rt = TensorRuntime(Comm(device=DEV), staleness=0).start(w, logic)
    for b in batches:
        rt.submit(b)
    out = rt.finish()
    tops = [e.value for e in out if isinstance(e, Left)]
    return w, tops


def test_online_mf_topk_fused_equals_torch_chains():
    """OnlineMFTopKWorker with the fused merge + SGD phases + index refresh against its
    torch chains: the first batch's top-K lists are identical (same index, same merge
    order), and after 6 batches of learning the item shard and the trained counts
    agree to fp32 atomic-order rounding.  (Without negatives: the known-item list the
    negatives are drawn from is appended by atomics, so two runs draw different
    negatives whichever path runs; with negatives the counts must still agree.)"""
    g = torch.Generator(device=DEV).manual_seed(3)
    users, items, B, D = 800, 4000, 512, 16
    batches = []
    for s in range(6):
        u = torch.randint(0, users, (B,), generator=g, device=DEV)
        u[:12] = 5  # repeated user: several occurrence rounds
        batches.append((u, torch.randint(0, items, (B,), generator=g, device=DEV),
                        torch.arange(B, device=DEV) + s * B, torch.rand(B, generator=g, device=DEV)))
    wf, tf = _run_online(True, batches, users, items, D)
    wt, tt = _run_online(False, batches, users, items, D)
    assert len(tf) == len(tt) == 6
    (_, s_f, i_f), (_, s_t, i_t) = tf[0], tt[0]
    assert torch.equal(i_f, i_t) and torch.equal(s_f, s_t)
    assert wf.trained == wt.trained == 6 * B
    torch.testing.assert_close(wf.items.weight, wt.items.weight, rtol=1e-4, atol=1e-5)
    # later batches: same lists up to near-ties moved by the rounding differences
    agree = sum(int((a[2] == b[2]).all(1).sum()) for a, b in zip(tf[1:], tt[1:]))
    assert agree >= 0.98 * 5 * B
    wf2, _ = _run_online(True, batches, users, items, D, neg=2)
    wt2, _ = _run_online(False, batches, users, items, D, neg=2)
    assert wf2.trained == wt2.trained > 6 * B
    assert bool(torch.isfinite(wf2.items.weight).all())


def test_online_learner_and_generator_gpu_matches_per_record():
    """The per-record parity of ``psOnlineLearnerAndGenerator`` (one rating per
    micro-batch, ``tests/test_topk_tensor.py``) on the GPU: fused merge, SGD phase
    kernels and index refresh give the reference's top-K lists."""
    import numpy as np

    from flink_parameter_server_1_amd.models.mf.apps import ps_online_learner_and_generator
    from flink_parameter_server_1_amd.models.mf.core import Rating
    from flink_parameter_server_1_amd.models.mf.pruning import LI
    from flink_parameter_server_1_amd.models.mf.topk_tensor import (as_reference_records,
                                                                    ps_online_learner_and_generator_tensor)
    from flink_parameter_server_1_amd.parallel.comm import Comm

    rng = np.random.default_rng(4)
    users, items, n, D = 12, 40, 150, 5
    rated, ratings = {}, []
    for t in range(n):
        u = int(rng.integers(0, users))
        left = [i for i in range(items) if i not in rated.setdefault(u, set())]
        it = int(left[int(rng.integers(0, len(left)))])
        rated[u].add(it)
        ratings.append(Rating(u, it, float(rng.random()), t))
    kw = dict(num_factors=D, range_min=-0.3, range_max=0.3, learning_rate=0.2, user_memory=4, K=6, worker_k=6,
              seed=9)
    ref_all = ps_online_learner_and_generator(ratings, bucket_size=8, pruning_algorithm=LI(2, 1.2), pull_limit=1,
                                              worker_parallelism=1, ps_parallelism=1, init="hash", **kw)
    batches = [(torch.tensor([r.user]), torch.tensor([r.item]), torch.tensor([r.timestamp]),
                torch.tensor([r.rating], dtype=torch.float32)) for r in ratings]
    out = ps_online_learner_and_generator_tensor(batches, users, items, bucket_size=8, pruning_algorithm=LI(2, 1.2),
                                                 comm=Comm(device=DEV), **kw)
    got = as_reference_records(out)
    assert len(got) == len(ref_all) == n
    for (u, it, ts, lst), (ru, rit, rts, rlst) in zip(got, ref_all):
        assert (u, it, ts) == (ru, rit, rts)
        assert [x[1] for x in lst] == [x[1] for x in rlst], ts
        np.testing.assert_allclose([x[0] for x in lst], [x[0] for x in rlst], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B", [1, 5, 64, 1000, 3000, 4096, 4097, 70_000])
def test_round_plan_kernel_equals_torch_plan(B):
    """``ops.round_plan`` (one workgroup after the sort) == the torch form of the fused
    RoundPlan, including long runs across thread chunks."""
    g = torch.Generator(device=DEV).manual_seed(B)
    users = torch.randint(0, max(2, B // 3), (B,), device=DEV, generator=g)
    if B > 100:
        users[: B // 2] = 17  # one run covering many chunks
    by_user, rnd, first, nu = ops.round_plan(users)
    ref = RoundPlan(users.cpu(), fused=True)  # the torch path (CPU)
    assert torch.equal(by_user.cpu(), ref.by_user)
    assert torch.equal(rnd.cpu(), ref.rnd) and torch.equal(first.cpu(), ref.first) and torch.equal(nu.cpu(), ref.nu)
