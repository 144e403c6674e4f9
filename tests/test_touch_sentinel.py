"""Untouched-row sentinel (``ShardedTable(touch_sentinel=True)``): zero-init additive
shards track the rows to dump at close by a -0.0 "never touched" value instead of a
byte of marks per row (``csrc/kernels/table_ops.hip``).  The dump must equal the
byte-mark bookkeeping's: every pulled row (also when its delta is zero or -0.0) and
every pushed row, nothing else; values read as plain zeros."""
import pytest
import torch

from flink_parameter_server_1_amd.parallel.table import ShardedTable

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _pair(device, n=1000, dim=3, world=1, rank=0, partition="range"):
    a = ShardedTable(n, dim, rank, world, partition, ("zeros",), 0, device, optimizer="add", touch_sentinel=True)
    b = ShardedTable(n, dim, rank, world, partition, ("zeros",), 0, device, optimizer="add")
    assert a.sentinel and a.touched is None and b.touched is not None
    return a, b


@pytest.mark.parametrize("device", DEVICES)
def test_sentinel_dump_equals_byte_marks(device):
    a, b = _pair(device)
    g = torch.Generator().manual_seed(0)
    for step in range(4):
        pull = torch.randint(0, 1000, (200,), generator=g, dtype=torch.int32).to(device)
        ra, rb = a.serve_rows(pull), b.serve_rows(pull)
        assert torch.equal(ra, rb)  # -0.0 == 0.0: reads as zeros
        push = torch.randint(0, 1000, (50,), generator=g, dtype=torch.int32).to(device)  # some never pulled
        d = torch.randn(50, 3, generator=g).to(device)
        d[::5] = -0.0  # a -0.0 delta still marks the row
        a.apply_rows(push, d, op="add")
        b.apply_rows(push, d, op="add")
    ia, va = a.dump()
    ib, vb = b.dump()
    assert torch.equal(ia, ib) and torch.equal(va, vb)
    assert not torch.signbit(va[va == 0]).any()  # dumped zeros are +0.0
    # mask, unserved rows untouched
    assert int(a.touched_mask().sum()) == ia.numel() < 1000


@pytest.mark.parametrize("device", DEVICES)
def test_sentinel_survives_snapshot_round_trip(device, tmp_path):
    from flink_parameter_server_1_amd.utils.io import restore_table, save_table

    a, _ = _pair(device)
    a.serve_rows(torch.tensor([3, 7, 11], dtype=torch.int32, device=device))
    a.apply_rows(torch.tensor([7, 500], dtype=torch.int32, device=device), torch.ones(2, 3, device=device))
    save_table(a, str(tmp_path / "t.shard0-of-1.bin"), only_touched=False)
    c, _ = _pair(device)
    restore_table(c, str(tmp_path / "t.shard*-of-*.bin"))
    ia, va = a.dump()
    ic, vc = c.dump()
    assert ia.tolist() == [3, 7, 11, 500] and torch.equal(ia, ic) and torch.equal(va, vc)


def test_sentinel_rejects_non_additive_or_nonzero_init():
    with pytest.raises(ValueError):
        ShardedTable(10, 2, init=("uniform", 0, 1), touch_sentinel=True)
    with pytest.raises(ValueError):
        ShardedTable(10, 2, init=("zeros",), optimizer="set", touch_sentinel=True)


@pytest.mark.parametrize("device", DEVICES)
def test_pa_paths_dump_the_pulled_features(device):
    """PA in place (the kernel flips first-pulled features) and through the PS path
    dump the same feature set: every feature of a trained example, also those whose
    update was zero (loss 0), as the reference's RangePSLogicWithClose (entries are
    created by the first pull)."""
    from flink_parameter_server_1_amd.models.pa.fast import DistributedPA, PAConfig, synthetic_sparse_batch
    from flink_parameter_server_1_amd.parallel.comm import Comm

    F = 1 << 16
    out = []
    for direct in (True, False):
        m = DistributedPA(PAConfig(feature_count=F, kind="binary", local_direct=direct),
                          Comm(device=torch.device(device)))
        feats = set()
        for s in range(4):
            ip, idx, val, lab = synthetic_sparse_batch(256, 16, F, seed=1, step=s, device=device)
            m.train_step(ip, idx, val, lab)
            feats |= set(idx.cpu().tolist())
        ids, w = m.dump()
        assert set(ids.cpu().tolist()) == feats
        o = torch.argsort(ids)
        out.append((ids[o].cpu(), w[o].reshape(-1).cpu()))
    assert torch.equal(out[0][0], out[1][0])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["binary", "multi"])
def test_sentinel_flip_never_clobbers_a_concurrent_add(kind):
    """the PA kernels flip a first-pulled feature's -0.0 sentinel in the
    table while other waves already add their updates into it.  Many examples share ONE
    fresh feature; the pulled snapshot stays -0.0 so every wave sees the sentinel and
    flips.  The table must hold the exact sum of the updates (a plain +0.0 store would
    drop every add that landed before it)."""
    from flink_parameter_server_1_amd import ops

    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(3)
    B, nnz, F, L = 8192, 8, 4096, 4
    idx = torch.randint(1, F, (B, nnz), generator=g)
    idx[:, 0] = 0  # the shared fresh feature
    ip = (torch.arange(B + 1) * nnz).long().to(dev)
    pos = idx.reshape(-1).to(torch.int32).to(dev)
    val = (torch.rand(B * nnz, generator=g) + 0.5).to(dev)
    if kind == "binary":
        y = (torch.randint(0, 2, (B,), generator=g) * 2 - 1).to(torch.int8).to(dev)
        snap = torch.full((F,), -0.0, device=dev)
        table = torch.full((F,), -0.0, device=dev)
        ref = torch.zeros(F, device=dev)
        ops.pa_binary(ip, val, pos, snap, y, "PA-I", 1.0, table, flip=table)
        ops.pa_binary(ip, val, pos, torch.zeros(F, device=dev), y, "PA-I", 1.0, ref)
    else:
        y = torch.randint(0, L, (B,), generator=g).to(torch.int32).to(dev)
        snap = torch.full((F, L), -0.0, device=dev)
        table = torch.full((F, L), -0.0, device=dev)
        ref = torch.zeros(F, L, device=dev)
        ops.pa_multi(ip, val, pos, snap, y, "ova", "PA-I", 1.0, None, table, flip=table)
        ops.pa_multi(ip, val, pos, torch.zeros(F, L, device=dev), y, "ova", "PA-I", 1.0, None, ref)
    torch.cuda.synchronize()
    assert (table[0].reshape(-1).view(torch.int32) != -(1 << 31)).all()  # no sentinel left on the shared feature
    torch.testing.assert_close(table + 0.0, ref, rtol=1e-4, atol=1e-4)
