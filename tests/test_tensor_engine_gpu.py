"""Tensor engine on the MI355X: the public batched API running the HIP kernels
(dedup, gather, fused MF SGD, apply incl. add_renorm, lock kernels)."""
import numpy as np
import pytest
import torch

from flink_parameter_server_1_amd import ops
from flink_parameter_server_1_amd.core.messages import Left, Right
from flink_parameter_server_1_amd.core.tensor_engine import TensorRuntime, fold_outputs
from flink_parameter_server_1_amd.models.mf.apps import ps_online_mf
from flink_parameter_server_1_amd.models.mf.core import Rating

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def test_native_library_loaded():
    assert ops.native_available()


def test_tensor_mf_gpu_matches_per_record_engine():
    """One rating per micro-batch on the GPU kernels (fp32) == per-record psOnlineMF
    (fp64, pullLimit 1, init='hash') to fp32 rounding."""
    from flink_parameter_server_1_amd.models.mf.batched import ps_online_mf_tensor
    from flink_parameter_server_1_amd.parallel.comm import Comm

    rng = np.random.default_rng(3)
    n, users, items = 200, 16, 24
    u, i, r = rng.integers(0, users, n), rng.integers(0, items, n), rng.random(n)
    kw = dict(num_factors=8, range_min=0.0, range_max=0.3, learning_rate=0.05, seed=11)
    recs = [Rating(int(a), int(b), float(c), t) for t, (a, b, c) in enumerate(zip(u, i, r))]
    Ur = {}
    Vr = {}
    for e in ps_online_mf(recs, init="hash", pull_limit=1, worker_parallelism=1, ps_parallelism=1, **kw):
        (Ur if e.is_left else Vr)[e.value[0]] = np.asarray(e.value[1])
    batches = [(torch.tensor(u[k:k + 1], device=DEV), torch.tensor(i[k:k + 1], device=DEV),
                torch.tensor(r[k:k + 1], dtype=torch.float32, device=DEV)) for k in range(n)]
    out = ps_online_mf_tensor(batches, users, items, comm=Comm(device=DEV), **kw)
    U, V = fold_outputs(out)
    assert set(U) == set(Ur) and set(V) == set(Vr)
    for k in Ur:
        np.testing.assert_allclose(U[k], Ur[k], rtol=0, atol=2e-6)
    for k in Vr:
        np.testing.assert_allclose(V[k], Vr[k], rtol=0, atol=2e-6)


def test_pipelined_engine_issues_no_implicit_sync():
    """staleness 1: counts reach the host one micro-batch ahead; no implicit
    device->host sync in the loop (torch sync-debug mode 'error')."""
    from flink_parameter_server_1_amd.models.mf.batched import OnlineMFWorker
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogicWithClose

    g = torch.Generator(device=DEV).manual_seed(0)
    users, items, B = 5000, 2000, 4096

    def batch():
        return (torch.randint(0, users, (B,), generator=g, device=DEV),
                torch.randint(0, items, (B,), generator=g, device=DEV),
                torch.rand(B, generator=g, device=DEV))

    rt = TensorRuntime(Comm(device=DEV), staleness=1)
    rt.start(OnlineMFWorker(users, 32, 0.05, emit_users=False),
             DeviceSimplePSLogicWithClose(items, 32, init=("uniform", 0.0, 0.1)))
    for _ in range(4):  # warm-up: workspaces allocated
        rt.submit(batch())
    data = [batch() for _ in range(20)]
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for b in data:
            rt.submit(b)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    rt.finish()
    ps = rt.ps_logic.ps
    assert ps.stats["steps"] == 24 and ps.stats["pulls"] == 24 * B


def test_pipelined_mf_topk_worker_syncs_once_per_batch():
    """OnlineMFTopKWorker (online MF + top-K serving) on the pipelined engine: the
    occurrence rounds of a batch's users are planned when it is received
    (``RoundPlan``) and the PS plans one batch ahead, so the only device->host sync
    left per micro-batch is the top-K scan's exactness certificate (did any query
    pass more candidates than the merge holds? then rescan unfused) -- at most one
    per batch, whatever the repeats of a user inside the batch."""
    import warnings

    from flink_parameter_server_1_amd.models.mf.topk_tensor import OnlineMFTopKWorker
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogic

    g = torch.Generator(device=DEV).manual_seed(0)
    users, items, B, D = 3000, 5000, 512, 16
    batches = []
    for s in range(20):
        u = torch.randint(0, users, (B,), generator=g, device=DEV)
        u[:8] = 7  # one user rated several times in the batch: several merge rounds
        batches.append((u, torch.randint(0, items, (B,), generator=g, device=DEV),
                        torch.arange(B, device=DEV) + s * B, torch.rand(B, generator=g, device=DEV)))
    w = OnlineMFTopKWorker(items, D, 0.01, K=20, worker_k=20, memory=64, negative_sample_rate=2,
                           prefill_items=True, num_users=users, resort_every=1000)
    logic = DeviceSimplePSLogic(users, D, op="add_renorm", init=("uniform", -0.01, 0.01))
    rt = TensorRuntime(Comm(device=DEV), staleness=1).start(w, logic)
    for b in batches[:4]:
        rt.submit(b)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("warn")
    try:
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            for b in batches[4:]:
                rt.submit(b)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    syncs = [r for r in rec if "synchroniz" in str(r.message)]
    assert len(syncs) <= 16, [str(r.message)[:120] for r in syncs]
    out = rt.finish()
    tops = [e.value for e in out if isinstance(e, Left)]
    assert len(tops) == 20
    (u0, _, _), S0, I0 = tops[-1]
    assert S0.shape == (B, 20) and bool((I0[:, 0] >= 0).all())


@pytest.mark.parametrize("dedup", [None, False])
def test_pipelined_pa_worker_issues_no_implicit_sync(dedup):
    """PAWorker on the pipelined engine (staleness 1): labelled and unlabelled
    examples mixed in every micro-batch, predictions emitted as MaskedPairs --
    no implicit device->host sync in the loop; the outputs compact when read."""
    from flink_parameter_server_1_amd.models.pa.batched import PAWorker
    from flink_parameter_server_1_amd.models.pa.fast import synthetic_sparse_batch
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceRangePSLogicWithClose

    F, B = 100_000, 2048
    batches = []
    for s in range(24):
        ip, idx, val, lab = synthetic_sparse_batch(B, 16, F, seed=1, step=s, device=DEV)
        lab = torch.where(torch.arange(B, device=DEV) % 4 == 0, torch.zeros_like(lab), lab)  # 1/4 unlabelled
        batches.append((ip, idx, val, lab))
    rt = TensorRuntime(Comm(device=DEV), staleness=1)
    rt.start(PAWorker("binary", 1, "PA", 1.0), DeviceRangePSLogicWithClose(F, 1, init=("zeros",), dedup=dedup))
    for b in batches[:4]:  # warm-up: workspaces allocated
        rt.submit(b)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for b in batches[4:]:
            rt.submit(b)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    out = rt.finish()
    preds = [e.value for e in out if isinstance(e, Left)]
    assert len(preds) == 24 and all(ids.numel() == B // 4 for ids, _ in preds)


def test_add_renorm_kernel_matches_reference():
    from flink_parameter_server_1_amd.ops import reference as R

    torch.manual_seed(0)
    for D in (8, 64, 100):
        T = torch.randn(300, D, device=DEV)
        st = T.norm(dim=1)
        idx = torch.randperm(300, device=DEV)[:120].to(torch.int32)
        idx[::7] = -1  # padding rows
        d = torch.randn(120, D, device=DEV)
        Tc, stc = T.cpu().clone(), st.cpu().clone()
        ops.apply_rows(T, idx, d, "add_renorm", state=st)
        R.apply_rows(Tc, idx.cpu(), d.cpu(), "add_renorm", state=stc)
        torch.testing.assert_close(T.cpu(), Tc, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(st.cpu(), stc, rtol=1e-5, atol=1e-6)


def test_lock_logic_gpu_no_lost_updates():
    from flink_parameter_server_1_amd.api.batched import BatchedWorkerLogic
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceLockPSLogic

    class W(BatchedWorkerLogic):
        def on_recv_batch(self, batch, ps):
            ps.pull(batch)

        def on_pull_recv_batch(self, pulled, ps):
            ps.push(pulled.values() + 1.0)

    rt = TensorRuntime(Comm(device=DEV)).start(W(), DeviceLockPSLogic(64, 4, op="set"))
    keys = torch.tensor([0, 0, 0, 5, 9, 9], device=DEV)
    for _ in range(5):
        rt.submit(keys)
    out = rt.finish()
    w = rt.ps_logic.table.weight.cpu()
    assert torch.equal(w[0], torch.full((4,), 15.0)) and torch.equal(w[9], torch.full((4,), 10.0))
    assert torch.equal(w[5], torch.full((4,), 5.0)) and float(w[1].abs().sum()) == 0.0
    assert sum(1 for e in out if isinstance(e, Right)) > 0


def test_model_load_and_double_load_gpu():
    from flink_parameter_server_1_amd.api.batched import BatchedWorkerLogic
    from flink_parameter_server_1_amd.core.tensor_engine import transform_tensor_with_double_model_load
    from flink_parameter_server_1_amd.core.messages import Left
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogicWithClose

    class W(BatchedWorkerLogic):
        def open(self, ctx):
            self.local = {}

        def update_model_batch(self, ids, values):
            for k, v in zip(ids.tolist(), values.reshape(-1).tolist()):
                self.local[k] = v

        def on_recv_batch(self, batch, ps):
            ps.pull(batch)

        def on_pull_recv_batch(self, pulled, ps):
            ps.push(torch.ones(len(pulled), 1, device=DEV))

        def close(self, ps):
            ps.output(dict(self.local))

    model = [Left((k, [10.0 * k])) for k in range(50)] + [Right((k, [float(-k)])) for k in range(5)]
    batches = [torch.arange(50, device=DEV) for _ in range(3)]
    out = transform_tensor_with_double_model_load(model, batches, W(), DeviceSimplePSLogicWithClose(50, 1),
                                                  comm=Comm(device=DEV))
    worker_local = [e.value for e in out if not isinstance(e, Right)][0]
    assert worker_local == {k: float(-k) for k in range(5)}
    ids, vals = [e.value for e in out if isinstance(e, Right)][0]
    got = dict(zip(ids.tolist(), vals.reshape(-1).tolist()))
    assert got == {k: 10.0 * k + 3 for k in range(50)}


def test_offline_mf_tensor_gpu_reaches_reference_rmse():
    """PSOfflineMatrixFactorizationTest on the GPU tensor engine: 100 java.util.Random(47)
    ratings, rank 15, 10 epochs with device shuffles, EOF-started replay -> RMSE <= 0.5."""
    from test_mf import reference_offline_ratings

    from flink_parameter_server_1_amd.models.mf.batched import ps_offline_mf_tensor
    from flink_parameter_server_1_amd.parallel.comm import Comm

    ratings = reference_offline_ratings()
    u = torch.tensor([x.user for x in ratings], device=DEV)
    i = torch.tensor([x.item for x in ratings], device=DEV)
    r = torch.tensor([x.rating for x in ratings], dtype=torch.float32, device=DEV)
    batches = [(u[s:s + 10], i[s:s + 10], r[s:s + 10]) for s in range(0, len(ratings), 10)]
    out = ps_offline_mf_tensor(batches, 20, 15, num_factors=15, range_min=0.0, range_max=1.0, learning_rate=0.01,
                               iterations=10, micro_batch=10, seed=3, comm=Comm(device=DEV))
    U, V = fold_outputs(out)
    err = np.sqrt(np.mean([(float(np.dot(U[x.user], V[x.item])) - x.rating) ** 2 for x in ratings]))
    assert err <= 0.5, err


def _counting_worker():
    from flink_parameter_server_1_amd.api.batched import FunctionBatchedWorkerLogic

    return FunctionBatchedWorkerLogic(lambda keys, ps: ps.pull(keys),
                                      lambda pulled, ps: ps.push(torch.ones(len(pulled), 4, device=DEV)))


@pytest.mark.parametrize("n", [20, 200])
def test_static_plans_apply_and_dump_only_real_keys(n):
    """World-1 static plans: n < key space pads the unique keys (padding gathers row 0),
    n >= key space takes the identity plan (every key served, presence flags).
    Either way only the requested keys are applied and enter the close-time dump."""
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogicWithClose

    g = torch.Generator(device=DEV).manual_seed(n)
    logic = DeviceSimplePSLogicWithClose(100, 4)
    rt = TensorRuntime(Comm(device=DEV), staleness=0).start(_counting_worker(), logic)
    assert logic.ps.identity_for(n) == (n >= 100)
    keys = [torch.randint(50, 90, (n,), generator=g, device=DEV) for _ in range(3)]
    for k in keys:
        rt.submit(k)
    out = rt.finish()
    ids, rows = out[-1].value
    allk = torch.cat(keys)
    want = torch.bincount(allk, minlength=100).float()
    assert sorted(ids.tolist()) == sorted(set(allk.tolist()))  # row 0 (padding) / absent keys not dumped
    torch.testing.assert_close(logic.table.weight[:, 0], want)


def test_mf_ps_identity_plan_matches_dedup_plan():
    """MF through the PS protocol with batches covering the item space: the identity
    plan (partition staged at receive time, pulled row = item id) trains like the
    de-duplicating plan."""
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    res = []
    for identity in (True, False):
        cfg = MFConfig(num_users=20000, num_items=1000, dim=64, learning_rate=0.05, force_ps_path=True, seed=3)
        m = DistributedMF(cfg, Comm(device=DEV))
        if not identity:
            m.ps.identity_for = lambda n: False
        data = SyntheticRatings(cfg.num_users, cfg.num_items, 1 << 18, device=DEV, truth_dim=8)
        for s in range(12):
            m.step(*data.batch(s, 1 << 15))
        m.flush()
        uid, iid, r = data.batch(0, 1 << 16)
        res.append((m.rmse(uid, iid, r), m.I.clone()))
    (r1, I1), (r0, I0) = res
    assert abs(r1 - r0) < 1e-3 * r0, (r1, r0)
    torch.testing.assert_close(I1, I0, rtol=1e-2, atol=1e-3)  # user rows are Hogwild across workgroups


def test_mf_ps_world1_fused_push_equals_delta_mode():
    """World 1, identity plans: the tiled SGD updating the served shard in place (the
    push applied by the kernel: no delta buffer, second row read or apply pass) trains
    the same model as the delta-mode kernel + pushed deltas.  The GPU step is not
    bit-deterministic (concurrent user-row reads see other deltas or not), so the
    fused run is compared with one delta-mode run at the distance between two
    delta-mode runs."""
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    res = []
    for fuse in (True, False, False):
        cfg = MFConfig(num_users=20000, num_items=1000, dim=64, learning_rate=0.05, force_ps_path=True, seed=3,
                       fuse_local_push=fuse, user_update="atomic", user_phases=2)
        m = DistributedMF(cfg, Comm(device=DEV))
        calls = []
        orig = m._item_sgd_in_place
        m._item_sgd_in_place = lambda *a: (calls.append(1), orig(*a))
        data = SyntheticRatings(cfg.num_users, cfg.num_items, 1 << 18, device=DEV, truth_dim=8)
        for s in range(12):
            m.step(*data.batch(s, 1 << 15))
        m.flush()
        assert bool(calls) == fuse
        uid, iid, r = data.batch(0, 1 << 16)
        res.append((m.rmse(uid, iid, r), m.I.clone(), m.U.clone(), m.ps.stats["pushes"]))
    (rf, If, Uf, pf), (r0, I0, U0, p0), (r1, I1, U1, p1) = res
    assert pf == p0 == p1 > 0
    noise_i = float((I1 - I0).abs().max())
    noise_u = float((U1 - U0).abs().max())
    assert float((If - I0).abs().max()) <= 3 * noise_i + 1e-6, (float((If - I0).abs().max()), noise_i)
    assert float((Uf - U0).abs().max()) <= 3 * noise_u + 1e-6, (float((Uf - U0).abs().max()), noise_u)
    assert abs(rf - r0) < 1e-3 * r0, (rf, r0)
