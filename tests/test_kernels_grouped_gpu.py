"""Item-grouped MF SGD kernel + counting-sort grouper vs the sequential fp32 reference."""
import pytest
import torch

from flink_parameter_server_1_amd import ops
from flink_parameter_server_1_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_csr_grouper_is_a_counting_sort():
    keys = torch.randint(0, 777, (20000,), dtype=torch.int32)
    g = ops.CSRGrouper(DEV)
    for _ in range(2):
        ptr, order = g.run(keys.to(DEV), 777)
        ptr_r, _ = R.csr_group(keys, 777)
        assert torch.equal(ptr.cpu(), ptr_r)
        o = order.cpu().long()
        assert torch.equal(torch.sort(o).values, torch.arange(keys.numel()))
        k_sorted = keys[o]
        assert bool((k_sorted[1:] >= k_sorted[:-1]).all())
        keys = torch.randint(0, 777, (15000,), dtype=torch.int32)


@pytest.mark.parametrize("D", [8, 15, 64, 100])
@pytest.mark.parametrize("mode", ["local", "pulled_f32", "pulled_bf16"])
def test_mf_sgd_grouped_matches_sequential(D, mode):
    """Unique users -> no Hogwild; items repeat, so the per-item sequential order matters
    and is checked exactly (the reference replays the kernel's own grouping order)."""
    nu, ni, B = 3000, 40, 1500
    torch.manual_seed(D)
    U = torch.rand(nu, D, device=DEV) * 0.3
    I = torch.rand(ni, D, device=DEV) * 0.3
    if mode == "pulled_bf16":
        I = I.to(torch.bfloat16)
    uid = torch.randperm(nu, device=DEV)[:B].to(torch.int32)
    iid = torch.randint(0, ni, (B,), device=DEV, dtype=torch.int32)
    r = torch.rand(B, device=DEV)
    ptr, order = ops.CSRGrouper(DEV).run(iid, ni)
    Ur, Ir = U.cpu().clone(), I.cpu().float().clone()
    delta = None if mode == "local" else torch.empty(ni, D, device=DEV)
    delta_r = None if mode == "local" else torch.empty(ni, D)
    R.mf_sgd_grouped(Ur, Ir, uid.cpu(), r.cpu(), ptr.cpu(), order.cpu(), 0.05, 0.01, delta_r)
    ops.mf_sgd_grouped(U, I, uid, r, ptr, order, 0.05, 0.01, delta)
    torch.testing.assert_close(U.cpu(), Ur, rtol=1e-4, atol=1e-5)
    if mode == "local":
        torch.testing.assert_close(I.cpu(), Ir, rtol=1e-4, atol=1e-5)
    else:
        torch.testing.assert_close(delta.cpu(), delta_r, rtol=1e-3, atol=1e-5)


def test_distributed_mf_grouped_vs_flat_converge():
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    res = {}
    for mode in ("grouped", "flat", "tiled"):  # tiled + force_ps_path: tile-grouped SGD on the pulled rows
        for force in (False, True):
            cfg = MFConfig(num_users=5000, num_items=800, dim=16, learning_rate=0.1, range_min=0.0, range_max=0.3,
                           sgd_mode=mode, force_ps_path=force, wire_dtype="bf16" if force else "fp32")
            m = DistributedMF(cfg, Comm(device=torch.device(DEV)))
            data = SyntheticRatings(5000, 800, 200000, device=DEV, truth_dim=4)
            uid, iid, r = data.batch(0, 200000)
            before = m.rmse(uid, iid, r)
            for s in range(60):
                m.step(*data.batch(s, 20000))
            res[(mode, force)] = (before, m.rmse(uid, iid, r))
    for k, (b, a) in res.items():
        assert a < 0.5 * b, (k, b, a)
