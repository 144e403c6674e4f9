"""Numerics of the gfx950 HIP kernels against the plain-PyTorch fp32 reference (ops.reference)."""
import pytest
import torch

from flink_parameter_server_1_amd import ops
from flink_parameter_server_1_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_native_library_loaded():
    assert ops.native_available()


@pytest.mark.parametrize("D", [1, 7, 16, 64, 100, 300])
def test_init_rows_matches_reference(D):
    t = torch.empty(1000, D, device=DEV)
    ops.init_rows(t, 3, 8, -0.5, 0.25, seed=42)
    ref = R.init_rows(torch.empty(1000, D), 3, 8, -0.5, 0.25, 42)
    torch.testing.assert_close(t.cpu(), ref, rtol=0, atol=1e-6)


@pytest.mark.parametrize("D", [1, 8, 64, 130])
@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
def test_gather_rows(D, wire):
    tab = torch.randn(5000, D, device=DEV)
    idx = torch.randint(0, 5000, (777,), device=DEV, dtype=torch.int32)
    touched = torch.zeros(5000, dtype=torch.uint8, device=DEV)
    out = ops.gather_rows(tab, idx, out_dtype=wire, touched=touched)
    torch.testing.assert_close(out.float(), tab[idx.long()].to(wire).float())
    assert int(touched.sum()) == int(torch.unique(idx).numel())


@pytest.mark.parametrize("op", ["add", "set", "sgd"])
@pytest.mark.parametrize("D", [1, 16, 64])
def test_apply_rows(op, D):
    tab = torch.randn(300, D, device=DEV)
    idx = torch.randperm(300, device=DEV)[:100].to(torch.int32)  # unique for 'set'
    if op != "set":
        idx = torch.cat([idx, idx[:40]])
    delta = torch.randn(idx.numel(), D, device=DEV)
    ref = tab.cpu().clone()
    R.apply_rows(ref, idx.cpu(), delta.cpu(), op, lr=0.1)
    ops.apply_rows(tab, idx, delta, op, lr=0.1)
    torch.testing.assert_close(tab.cpu(), ref, rtol=1e-5, atol=1e-5)


# 16-byte kernels (D % 4 == 0, aligned): NV = 1 at D <= 256, 2 at 300, 4 at 520;
# D = 1028 and the misaligned view take the scalar kernels
@pytest.mark.parametrize("D", [1, 4, 64, 300, 520, 1028])
@pytest.mark.parametrize("misaligned", [False, True])
def test_gather_apply_v4_paths(D, misaligned):
    g = torch.Generator(device=DEV).manual_seed(D)
    base = torch.randn(3001 * D + 1, device=DEV, generator=g)
    tab = (base[1:] if misaligned else base[:-1]).view(3001, D)
    tab[::7] = -0.0  # sentinel rows: the gather flips served ones to +0.0
    idx = torch.randint(0, 3001, (1111,), device=DEV, dtype=torch.int32, generator=g)
    ref_tab = tab.clone()
    touched = torch.zeros(3001, dtype=torch.uint8, device=DEV)
    out = ops.gather_rows(tab, idx, touched=touched, flip=True)
    assert torch.equal(out, ref_tab[idx.long()])
    served = torch.zeros(3001, dtype=torch.bool, device=DEV)
    served[idx.long()] = True
    flipped = ref_tab.clone()
    flipped[served] = flipped[served] + 0.0  # -0.0 + 0.0 = +0.0
    assert torch.equal(tab.view(torch.int32), flipped.view(torch.int32))
    assert torch.equal(touched.bool(), served)
    uniq = torch.unique(idx)
    for op in ("add_unique", "set"):
        delta = torch.randn(uniq.numel(), D, device=DEV, generator=g)
        delta[::5] = -0.0
        ref = tab.cpu().clone()
        R.apply_rows(ref, uniq.cpu(), delta.cpu(), "add" if op == "add_unique" else "set")
        ops.apply_rows(tab, uniq, delta, op)
        assert torch.equal(tab.cpu(), ref)
        assert not torch.signbit(tab[uniq.long()][tab[uniq.long()] == 0]).any()  # -0.0 deltas leave +0.0


@pytest.mark.parametrize("D,out_dtype", [(64, torch.float32), (300, torch.float32), (7, torch.float32),
                                         (64, torch.bfloat16), (1, torch.float32), (1, torch.bfloat16)])
def test_gather_padding_slots_serve_zero_rows(D, out_dtype):
    """Fixed-shape plans pad with row -1: a zero row, no touched mark, no sentinel flip
    (16-byte, scalar and bf16-wire gathers) -- same as the torch twin."""
    tab = torch.randn(500, D, device=DEV)
    tab[::3] = -0.0
    idx = torch.randint(0, 500, (777,), device=DEV, dtype=torch.int32)
    idx[::4] = -1
    ref_tab, ref_touched = tab.cpu().clone(), torch.zeros(500, dtype=torch.uint8)
    touched = torch.zeros(500, dtype=torch.uint8, device=DEV)
    out = ops.gather_rows(tab, idx, out_dtype=out_dtype, touched=touched, flip=True)
    ref = R.gather_rows(ref_tab, idx.cpu(), out_dtype, ref_touched)
    ops.flip_sentinel(ref_tab, idx.cpu())
    # (as floats: a repeated sentinel row may be served before or after its flip, -0.0 or +0.0)
    assert torch.equal(out.cpu().float(), ref.float())
    assert torch.equal(out[::4].float(), torch.zeros_like(out[::4].float()))
    assert torch.equal(touched.cpu(), ref_touched)
    assert torch.equal(tab.cpu().view(torch.int32), ref_tab.view(torch.int32))
    marks = torch.zeros(500, dtype=torch.uint8, device=DEV)
    ops.mark_rows(marks, idx)
    assert torch.equal(marks.cpu(), ref_touched)


def test_apply_adagrad_bf16_delta():
    D = 64
    tab = torch.randn(200, D, device=DEV)
    state = torch.rand(200, D, device=DEV)
    idx = torch.randperm(200, device=DEV)[:64].to(torch.int32)
    delta = torch.randn(64, D, device=DEV).to(torch.bfloat16)
    ref_t, ref_s = tab.cpu().clone(), state.cpu().clone()
    R.apply_rows(ref_t, idx.cpu(), delta.cpu().float(), "adagrad", lr=0.05, state=ref_s)
    ops.apply_rows(tab, idx, delta, "adagrad", lr=0.05, state=state)
    torch.testing.assert_close(tab.cpu(), ref_t, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(state.cpu(), ref_s, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("method", ["claim", "flags"])
@pytest.mark.parametrize("W,kind,hashed,num_ids", [(1, 0, False, 10007), (3, 0, False, 10007), (8, 0, False, 10007),
                                                   (4, 1, False, 10007), (4, 1, False, 9), (3, 0, False, 300_000),
                                                   (1, 0, True, 10007), (8, 0, True, 2_000_000_011),
                                                   (4, 1, True, 2_000_000_011)])
def test_dedup(W, kind, hashed, num_ids, method):
    if hashed and method == "flags":
        pytest.skip("flags is a dense-map method")
    block = -(-num_ids // W)
    keys = torch.randint(0, num_ids, (50000,), dtype=torch.int32)
    if num_ids > 1_000_000:  # make duplicates likely in a huge id space
        keys = keys[torch.randint(0, 8000, (50000,))]
    ws = ops.DedupWorkspace(num_ids, W, kind, block, DEV, hashed=hashed, method=method)
    for it in range(3):  # epoch tagging: later calls must not see earlier ones; 3rd call grows the hash table
        counts, prefix, uniq, pos = ws.run(keys.to(DEV))
        c_ref, p_ref, u_ref, pos_ref = R.dedup(keys, W, kind, block)
        assert counts.cpu().tolist() == c_ref.tolist()
        assert prefix.cpu().tolist() == p_ref.tolist()
        U = int(prefix[-1])
        # same unique set per shard group, and every request points to its key
        for d in range(W):
            a, b = int(p_ref[d]), int(p_ref[d + 1])
            assert sorted(uniq[a:b].cpu().tolist()) == sorted(u_ref[a:b].tolist())
        _, local = R.shard_of(keys, W, kind, block)
        assert torch.equal(uniq[:U].cpu()[pos.cpu().long()].long(), local)
        keys = torch.randint(0, num_ids, (30000 if it == 0 else 90000,), dtype=torch.int32)
        if num_ids > 1_000_000:
            keys = keys[torch.randint(0, 5000, (keys.numel(),))]


@pytest.mark.parametrize("W,kind", [(1, 0), (3, 0), (4, 1), (5, 2)])
@pytest.mark.parametrize("hashed", [False, True])
def test_route_requests(W, kind, hashed):
    """Request plans (``DedupWorkspace.route``): every request is an entry of the
    shard-major ``uniq`` (no de-duplication), ``pos`` a permutation of the requests,
    the shard counts those of the reference grouping."""
    num_ids = 1 << 30 if hashed else 100_000
    block = -(-num_ids // W)
    ws = ops.DedupWorkspace(num_ids, W, kind, block, DEV, hashed=hashed)
    for n in (50000, 20000, 120000):  # the third call grows the workspace
        keys = torch.randint(0, num_ids, (n,), dtype=torch.int32)
        keys[: n // 4] = keys[n // 4: n // 2]  # repeated keys stay separate entries
        counts, prefix, uniq, pos = ws.route(keys.to(DEV))
        c_ref, p_ref, u_ref, _ = R.route(keys, W, kind, block)
        assert counts.cpu().tolist() == c_ref.tolist()
        assert prefix.cpu().tolist() == p_ref.tolist()
        assert int(prefix[-1]) == n
        p = pos.cpu().long()
        assert torch.equal(torch.sort(p).values, torch.arange(n))  # a permutation
        _, local = R.shard_of(keys, W, kind, block)
        assert torch.equal(uniq[:n].cpu()[p].long(), local)
        for d in range(W):  # every request sits in its owner's group
            a, b = int(p_ref[d]), int(p_ref[d + 1])
            dest, _ = R.shard_of(keys, W, kind, block)
            assert bool(((p >= a) & (p < b) == (dest == d)).all())


@pytest.mark.parametrize("D", [8, 15, 64, 128])
def test_mf_sgd_local_unique_rows(D):
    """Unique users/items per batch -> the Hogwild kernel is deterministic."""
    nu, ni, B = 4000, 3000, 2500
    U = torch.rand(nu, D, device=DEV) * 0.1
    I = torch.rand(ni, D, device=DEV) * 0.1
    uid = torch.randperm(nu, device=DEV)[:B].to(torch.int32)
    iid = torch.randperm(ni, device=DEV)[:B].to(torch.int32)
    r = torch.rand(B, device=DEV)
    Ur, Ir = U.cpu().clone(), I.cpu().clone()
    R.mf_sgd_local(Ur, Ir, uid.cpu(), iid.cpu(), r.cpu(), 0.05, 0.01)
    ops.mf_sgd_local(U, I, uid, iid, r, 0.05, 0.01)
    torch.testing.assert_close(U.cpu(), Ur, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(I.cpu(), Ir, rtol=1e-5, atol=1e-6)


def test_mf_sgd_local_duplicate_items_accumulate():
    D, B = 64, 4096
    # small user factors: the items' in-batch drift (Hogwild reads of rows
    # other ratings already updated) then only changes e at second order, so
    # the sum of the ~256 atomic adds per item must match the snapshot reference
    U = torch.rand(B, D, device=DEV) * 1e-3
    I = torch.rand(16, D, device=DEV) * 0.1
    uid = torch.arange(B, device=DEV, dtype=torch.int32)
    iid = torch.randint(0, 16, (B,), device=DEV, dtype=torch.int32)
    r = torch.rand(B, device=DEV)
    Ur, Ir = U.cpu().clone(), I.cpu().clone()
    R.mf_sgd_local(Ur, Ir, uid.cpu(), iid.cpu(), r.cpu(), 0.01)
    ops.mf_sgd_local(U, I, uid, iid, r, 0.01)
    torch.testing.assert_close(I.cpu(), Ir, rtol=1e-4, atol=1e-6)
    assert not torch.equal(I.cpu(), I.cpu() * 0)  # sanity


@pytest.mark.parametrize("wire", [torch.float32, torch.bfloat16])
def test_mf_sgd_pulled(wire):
    D, nu, B, NU = 64, 5000, 3000, 700
    U = torch.rand(nu, D, device=DEV) * 0.1
    uid = torch.randperm(nu, device=DEV)[:B].to(torch.int32)
    rows = (torch.rand(NU, D, device=DEV) * 0.1).to(wire)
    pos = torch.randint(0, NU, (B,), device=DEV, dtype=torch.int32)
    r = torch.rand(B, device=DEV)
    delta = torch.zeros(NU, D, device=DEV)
    Ur, dr = U.cpu().clone(), delta.cpu().clone()
    R.mf_sgd_pulled(Ur, uid.cpu(), r.cpu(), rows.cpu(), pos.cpu(), dr, 0.03)
    ops.mf_sgd_pulled(U, uid, r, rows, pos, delta, 0.03)
    torch.testing.assert_close(U.cpu(), Ur, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(delta.cpu(), dr, rtol=1e-4, atol=1e-6)


def test_mf_sq_err():
    D = 64
    U = torch.rand(1000, D, device=DEV)
    I = torch.rand(500, D, device=DEV)
    uid = torch.randint(0, 1000, (9999,), device=DEV, dtype=torch.int32)
    iid = torch.randint(0, 500, (9999,), device=DEV, dtype=torch.int32)
    r = torch.rand(9999, device=DEV) * 20
    got = float(ops.mf_sq_err(U, I, uid, iid, r).item())
    ref = R.mf_sq_err(U.cpu(), I.cpu(), uid.cpu(), iid.cpu(), r.cpu())
    assert abs(got - ref) / ref < 1e-5


@pytest.mark.parametrize("W", [2, 3, 8])
def test_rot_partition_matches_reference(W):
    from flink_parameter_server_1_amd.parallel.rotation import shard_halves

    NI, n = 100_003, 300_000
    half = torch.tensor(shard_halves(NI, W), dtype=torch.int32)
    uid = torch.randint(0, 10_000, (n,), dtype=torch.int32)
    iid = torch.randint(0, NI, (n,), dtype=torch.int32)
    r = torch.rand(n)
    c_ref, p_ref, u_ref, row_ref, r_ref = R.rot_partition(uid, iid, r, W, half)
    part = ops.RotationPartitioner(W, half, DEV)
    for _ in range(2):  # buffers / counters reused
        ptr, u, row, rr = part.run(uid.to(DEV), iid.to(DEV), r.to(DEV))
        assert ptr.cpu().tolist() == p_ref.tolist()
        for k in range(2 * W):  # order inside a block is arbitrary: compare as multisets of triples
            a, b = int(p_ref[k]), int(p_ref[k + 1])
            key = lambda U, Rw, Rt: sorted(zip(U[a:b].tolist(), Rw[a:b].tolist(), Rt[a:b].tolist()))  # noqa: E731
            assert key(u.cpu(), row.cpu(), rr.cpu()) == key(u_ref, row_ref, r_ref)


def test_mf_sgd_local_seg_matches_slice():
    D, nu, ni, B = 64, 5000, 4000, 3000
    U = torch.rand(nu, D, device=DEV) * 0.1
    I = torch.rand(ni, D, device=DEV) * 0.1
    uid = torch.randperm(nu, device=DEV)[:B].to(torch.int32)
    iid = torch.randperm(ni, device=DEV)[:B].to(torch.int32)
    r = torch.rand(B, device=DEV)
    ptr = torch.tensor([0, 1000, 2500, 3000], dtype=torch.int32, device=DEV)
    Ur, Ir = U.cpu().clone(), I.cpu().clone()
    R.mf_sgd_local(Ur, Ir, uid[1000:2500].cpu(), iid[1000:2500].cpu(), r[1000:2500].cpu(), 0.05, 0.01)
    ops.mf_sgd_local_seg(U, I, uid, iid, r, ptr, 1, B, 0.05, 0.01)
    torch.testing.assert_close(U.cpu(), Ur, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(I.cpu(), Ir, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("rec8", [False, True])
@pytest.mark.parametrize("phases", [1, 3])
@pytest.mark.parametrize("skew", [False, True])
@pytest.mark.parametrize("W,R", [(1, 128), (2, 64), (8, 64), (1, 256), (1, 16)])
def test_tile_partition_matches_reference(W, R, rec8, skew, phases):
    """(1, 16): 25k+ buckets -- the count kernel's 16-bit LDS counters; with skew,
    one workgroup counts ~60k ratings of a hot item (overflow-safe flushes)."""
    from flink_parameter_server_1_amd.parallel.rotation import block_rows, shard_halves

    NI, n = 200_003, 500_000
    half = [NI] if W == 1 else shard_halves(NI, W)
    rows_max = NI if W == 1 else max(block_rows(NI, W))
    T = -(-rows_max // R)
    half_t = torch.tensor(half, dtype=torch.int32)
    uid = torch.randint(0, 10_000, (n,), dtype=torch.int32)
    iid = torch.randint(0, NI, (n,), dtype=torch.int32)
    if skew:  # 70% of the ratings on 3 hot items: coarse keys of very different sizes
        hot = torch.tensor([5, NI // 2, NI - 1], dtype=torch.int32)
        iid = torch.where(torch.rand(n) < 0.7, hot[torch.randint(0, 3, (n,))], iid)
    r = torch.rand(n)
    upp = -(-10_000 // phases)
    if phases * 2 * W * T > ops.TILE_MAX_BUCKETS:
        pytest.skip("bucket count above the LDS counters")
    p_ref, u_ref, row_ref, r_ref = R_tile(uid, iid, r, W, half_t, R, T, phases, upp)
    part = ops.TilePartitioner(W, half, R, T, DEV, rec8=rec8, phases=phases, users_per_phase=upp)
    seen = torch.zeros(NI, dtype=torch.uint8, device=DEV)
    for _ in range(2):
        ptr, rec = part.run(uid.to(DEV), iid.to(DEV), r.to(DEV), seen)
        u, row, rr = part.unpack(rec, ptr)
        ptr_c = ptr.cpu()
        assert torch.equal(ptr_c, p_ref)
        # same multiset of (bucket, uid, row, rating): sort both by (bucket, uid, row)
        for t_ in (u, row, rr):
            assert t_.numel() == n
        bucket = torch.repeat_interleave(torch.arange(p_ref.numel() - 1), (p_ref[1:] - p_ref[:-1]).long())
        key = lambda U_, Rw, Rt: sorted(zip(bucket.tolist(), U_.tolist(), Rw.tolist(), Rt.tolist()))  # noqa: E731
        assert key(u.cpu(), row.cpu(), rr.cpu()) == key(u_ref, row_ref, r_ref)
    assert torch.equal(seen.cpu().bool(), torch.bincount(iid.long(), minlength=NI) > 0)


@pytest.mark.parametrize("rec8", [False, True])
@pytest.mark.parametrize("W,phases", [(1, 1), (8, 3)])
def test_tile_partition_drops_out_of_range_ids(W, phases, rec8):
    """Ratings whose user or item id lies outside the tables (negative, or at / past the
    bound) are dropped by the partition -- the count and level-1 passes skip them alike --
    instead of indexing past the bucket counters and, in the SGD, past the tables: the
    result equals the partition of the valid ratings alone."""
    from flink_parameter_server_1_amd.parallel.rotation import block_rows, shard_halves

    NI, NU, n, R = 50_003, 9_000, 300_000, 64
    half = [NI] if W == 1 else shard_halves(NI, W)
    T = -(-(NI if W == 1 else max(block_rows(NI, W))) // R)
    upp = -(-NU // phases)
    g = torch.Generator().manual_seed(W + phases)
    uid = torch.randint(0, NU, (n,), dtype=torch.int32, generator=g)
    iid = torch.randint(0, NI, (n,), dtype=torch.int32, generator=g)
    bad = torch.rand(n, generator=g)
    uid = torch.where(bad < 0.02, NU + (uid % 7), uid)          # past the user shard (inside the phases' range
    uid = torch.where((bad >= 0.02) & (bad < 0.03), -1 - uid % 5, uid)  # at phases * upp >= NU) / negative
    iid = torch.where((bad >= 0.03) & (bad < 0.05), NI + (iid % 11), iid)
    r = torch.rand(n, generator=g)
    keep = (uid >= 0) & (uid < NU) & (iid < NI)
    part = ops.TilePartitioner(W, half, R, T, DEV, rec8=rec8, phases=phases, users_per_phase=upp,
                               num_users=NU, num_items=NI)
    ptr, rec = part.run(uid.to(DEV), iid.to(DEV), r.to(DEV))
    p_ref, u_ref, row_ref, r_ref = R_tile(uid[keep], iid[keep], r[keep], W, torch.tensor(half, dtype=torch.int32), R,
                                          T, phases, upp)
    assert torch.equal(ptr.cpu(), p_ref) and int(p_ref[-1]) == int(keep.sum()) < n
    u, row, rr = part.unpack(rec[: int(p_ref[-1])], ptr)
    bucket = torch.repeat_interleave(torch.arange(p_ref.numel() - 1), (p_ref[1:] - p_ref[:-1]).long())
    key = lambda U_, Rw, Rt: sorted(zip(bucket.tolist(), U_.tolist(), Rw.tolist(), Rt.tolist()))  # noqa: E731
    assert key(u.cpu(), row.cpu(), rr.cpu()) == key(u_ref, row_ref, r_ref)


@pytest.mark.parametrize("W,R,skew", [(1, 128, True), (8, 64, False), (1, 16, True)])
def test_tile_partition_32bit_counters_match_reference(W, R, skew, monkeypatch):
    """The 32-bit counter path of the count kernel (``FPS_TP_H16=0``; 16-bit packed
    counters are the default at every bucket count): same partition as the reference."""
    monkeypatch.setenv("FPS_TP_H16", "0")
    try:
        test_tile_partition_matches_reference(W, R, True, skew, 3)
    finally:
        monkeypatch.delenv("FPS_TP_H16")
        N_lib().fps_tile_partition_set_h16(1)


@pytest.mark.parametrize("rec8", [False, True])
@pytest.mark.parametrize("W,R,skew,phases", [(1, 128, True, 3), (8, 64, False, 3), (2, 64, True, 1), (1, 256, False, 1)])
def test_tile_partition_slim_kernels_match_reference(W, R, skew, phases, rec8, monkeypatch):
    """The slim partition shape (``FPS_TP_SLIM=1``: 256-thread count / scatter workgroups,
    1024-record LDS batches, co-resident with the tile SGD): same partition as the
    reference, skewed coarse keys included."""
    prev = N_lib().fps_tile_partition_get_slim()
    monkeypatch.setenv("FPS_TP_SLIM", "1")
    try:
        test_tile_partition_matches_reference(W, R, rec8, skew, phases)
        assert N_lib().fps_tile_partition_get_slim() == 1
    finally:
        monkeypatch.delenv("FPS_TP_SLIM")
        N_lib().fps_tile_partition_set_slim(prev)


def N_lib():
    from flink_parameter_server_1_amd.ops import _native

    return _native.require()


def R_tile(*a):
    return R.tile_partition(*a)


@pytest.mark.parametrize("grid", [3, 40])
def test_tile_partition_capped_grid_loops_over_chunks(grid, monkeypatch):
    """FPS_TP_GRID caps every partition launch's workgroups: level-1 workgroups loop over
    the chunks, count workgroups take several chunks each -- same partition (per bucket,
    as a multiset) as the reference."""
    monkeypatch.setenv("FPS_TP_GRID", str(grid))
    try:
        NI, NU, R, n, P = 100_000, 200_000, 64, 1 << 23, 2  # 8M ratings: 32 level-1 chunks
        T = -(-NI // R)
        half_t = torch.tensor([NI], dtype=torch.int32)
        g = torch.Generator().manual_seed(grid)
        uid = torch.randint(0, NU, (n,), dtype=torch.int32, generator=g)
        iid = torch.randint(0, NI, (n,), dtype=torch.int32, generator=g)
        r = torch.rand(n, generator=g)
        upp = -(-NU // P)
        part = ops.TilePartitioner(1, [NI], R, T, DEV, rec8=True, phases=P, users_per_phase=upp)
        ptr, rec = part.run(uid.to(DEV), iid.to(DEV), r.to(DEV))
        p_ref, u_ref, row_ref, r_ref = R_tile(uid, iid, r, 1, half_t, R, T, P, upp)
        assert torch.equal(ptr.cpu(), p_ref)
        u, row, rr = part.unpack(rec, ptr)
        bucket = torch.repeat_interleave(torch.arange(p_ref.numel() - 1), (p_ref[1:] - p_ref[:-1]).long())
        def canon(b, uu, ro, ra):  # lexicographic (bucket, user, row, rating bits) order
            hi = (b.long() * (1 << 21) + uu.long()) * 256 + ro.long()
            bits = ra.float().view(torch.int32).long()
            o = torch.argsort(bits, stable=True)
            o = o[torch.argsort(hi[o], stable=True)]
            return hi[o], bits[o]

        gh, gb = canon(bucket, u.cpu(), row.cpu(), rr.cpu())
        wh, wb = canon(bucket, u_ref, row_ref, r_ref)
        assert torch.equal(gh, wh) and torch.equal(gb, wb)
    finally:
        from flink_parameter_server_1_amd.ops import _native

        _native.require().fps_tile_partition_set_grid(0)


def test_tile_partition_16bit_counters_survive_one_hot_bucket():
    """Every rating on ONE item: one bucket gets all n = 1M counts, four times the
    16-bit range per count workgroup -- the flushes must keep the counts exact."""
    NI, R, n = 200_003, 16, 1 << 20
    T = -(-NI // R)
    assert ops.TILE_MAX_BUCKETS >= 2 * T > 16384  # the 16-bit counter path
    uid = torch.randint(0, 5000, (n,), dtype=torch.int32)
    iid = torch.full((n,), 12345, dtype=torch.int32)
    iid[::97] = torch.randint(0, NI, (iid[::97].numel(),), dtype=torch.int32)
    r = torch.rand(n)
    half_t = torch.tensor([NI], dtype=torch.int32)
    p_ref, u_ref, row_ref, r_ref = R_tile(uid, iid, r, 1, half_t, R, T, 1, 5000)
    part = ops.TilePartitioner(1, [NI], R, T, DEV, rec8=True, phases=1, users_per_phase=5000)
    ptr, rec = part.run(uid.to(DEV), iid.to(DEV), r.to(DEV))
    assert torch.equal(ptr.cpu(), p_ref)
    u, row, rr = part.unpack(rec, ptr)
    bucket = torch.repeat_interleave(torch.arange(p_ref.numel() - 1), (p_ref[1:] - p_ref[:-1]).long())
    got = sorted(zip(bucket.tolist(), u.cpu().tolist(), row.cpu().tolist(), rr.cpu().tolist()))
    want = sorted(zip(bucket.tolist(), u_ref.tolist(), row_ref.tolist(), r_ref.tolist()))
    assert got == want


@pytest.mark.parametrize("rec8", [False, True])
@pytest.mark.parametrize("D", [16, 32, 64, 128, 256])
def test_mf_sgd_tiled_unique_rows(D, rec8):
    """Unique users and items: the tiled kernel equals the batch reference."""
    nu, ni, B = 6000, 5000, 3000
    U = torch.rand(nu, D, device=DEV) * 0.1
    I = torch.rand(ni, D, device=DEV) * 0.1
    uid = torch.randperm(nu, device=DEV)[:B].to(torch.int32)
    iid = torch.randperm(ni, device=DEV)[:B].to(torch.int32)
    r = torch.rand(B, device=DEV)
    Rt = ops.tile_rows_for(D, ni, 1)
    T = -(-ni // Rt)
    part = ops.TilePartitioner(1, [ni], Rt, T, DEV, rec8=rec8)  # one block: the whole table
    ptr, rec = part.run(uid, iid, r)
    Ur, Ir = U.cpu().clone(), I.cpu().clone()
    R.mf_sgd_local(Ur, Ir, uid.cpu(), iid.cpu(), r.cpu(), 0.05, 0.01)
    ops.mf_sgd_tiled(U, I, rec, ptr, 0, T, Rt, 0.05, 0.01)
    torch.testing.assert_close(U.cpu(), Ur, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(I.cpu(), Ir, rtol=1e-5, atol=1e-6)


def test_mf_sgd_tiled_user_modes_match_reference_rmw_and_atomic_sums():
    """User-row modes of the tiled kernel vs the fp32 reference: sc1 / atomic equal the
    plain kernel on unique users; with every user repeated 8 times in one launch the
    atomic mode (exact: float-atomic user deltas) equals the reference's summed user
    deltas (``R.mf_sgd_local(user_atomic=True)``), D = 16 / 64 / 128 (the lane transposition
    of the contiguous atomics at 4, 16 and 16 x 2 lanes per chunk)."""
    for D in (16, 64, 128):
        nu, ni, B = 6000, 5000, 3000
        U0 = torch.rand(nu, D, device=DEV) * 0.1
        I0 = torch.rand(ni, D, device=DEV) * 0.1
        uid = torch.randperm(nu, device=DEV)[:B].to(torch.int32)
        iid = torch.randperm(ni, device=DEV)[:B].to(torch.int32)
        r = torch.rand(B, device=DEV)
        Rt = ops.tile_rows_for(D, ni, 1)
        T = -(-ni // Rt)
        ptr, rec = ops.TilePartitioner(1, [ni], Rt, T, DEV, rec8=True).run(uid, iid, r)
        out = []
        for mode in (0, 1, 2):
            U, I = U0.clone(), I0.clone()
            ops.mf_sgd_tiled(U, I, rec, ptr, 0, T, Rt, 0.05, 0.01, user_mode=mode)
            out.append((U, I))
        for U, I in out[1:]:
            torch.testing.assert_close(U, out[0][0], rtol=1e-6, atol=1e-7)
            torch.testing.assert_close(I, out[0][1], rtol=1e-6, atol=1e-7)
        # repeated users, distinct items: users get 8 deltas each in one launch
        uid8 = (torch.arange(B, device=DEV) % (B // 8)).to(torch.int32)
        ptr, rec = ops.TilePartitioner(1, [ni], Rt, T, DEV, rec8=True).run(uid8, iid, r)
        # lr 0.01: a user's 8 ratings may read its row before or after the others' adds
        # landed -- second order in lr for the user rows (measured ~1e-4 at lr 0.05, D 128:
        # ~4e-6 here) and for the item rows (an item's delta is first order in the user row
        # it read, and that row's spread is first order: ~1e-5 here) -- while a LOST user
        # delta is first order, lr * |e| * max|i| ~ 3e-4
        lr = 0.01
        U, I = U0.clone(), I0.clone()
        ops.mf_sgd_tiled(U, I, rec, ptr, 0, T, Rt, lr, 0.0, user_mode=2)
        Ur, Ir = U0.cpu().clone(), I0.cpu().clone()
        R.mf_sgd_local(Ur, Ir, uid8.cpu(), iid.cpu(), r.cpu(), lr, 0.0, user_atomic=True)
        assert float((U.cpu() - Ur).abs().max()) < 3e-5, D
        assert float((I.cpu() - Ir).abs().max()) < 1e-4, D
        assert float((U.cpu() - U0.cpu()).abs().max()) > 3e-4  # the deltas did land


@pytest.mark.parametrize("rec8", [False, True])
def test_mf_sgd_tiled_pair_matches_two_launches(rec8):
    """Both item blocks in one launch (``mf_sgd_tiled_pair``): unique users and items,
    so it equals the batch reference; blocks of unequal size."""
    D, nu, ni, B = 64, 9000, 5001, 4000
    U = torch.rand(nu, D, device=DEV) * 0.1
    I = torch.rand(ni, D, device=DEV) * 0.1
    uid = torch.randperm(nu, device=DEV)[:B].to(torch.int32)
    iid = torch.randperm(ni, device=DEV)[:B].to(torch.int32)
    r = torch.rand(B, device=DEV)
    h0 = 2600
    Rt = ops.tile_rows_for(D, ni, 2)
    T = -(-h0 // Rt)
    ptr, rec = ops.TilePartitioner(1, [h0], Rt, T, DEV, rec8=rec8).run(uid, iid, r)
    Ur, Ir = U.cpu().clone(), I.cpu().clone()
    R.mf_sgd_local(Ur, Ir, uid.cpu(), iid.cpu(), r.cpu(), 0.05, 0.01)
    ops.mf_sgd_tiled_pair(U, I[:h0], I[h0:], rec, ptr, 0, T, Rt, 0.05, 0.01)
    torch.testing.assert_close(U.cpu(), Ur, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(I.cpu(), Ir, rtol=1e-5, atol=1e-6)


def test_mf_sgd_tiled_duplicate_items_accumulate():
    """Many ratings per item: LDS atomics must keep every item delta (no lost update)."""
    D, B, ni = 64, 20000, 300
    nu = B
    U = torch.full((nu, D), 1e-3, device=DEV)
    I = torch.rand(ni, D, device=DEV) * 0.1
    uid = torch.arange(B, device=DEV, dtype=torch.int32)
    iid = torch.randint(0, ni, (B,), device=DEV, dtype=torch.int32)
    r = torch.rand(B, device=DEV)
    Rt = 64
    T = -(-ni // Rt)
    ptr, rec = ops.TilePartitioner(1, [ni], Rt, T, DEV).run(uid, iid, r)  # ~67 ratings per row, 4.3k per tile
    Ur, Ir = U.cpu().clone(), I.cpu().clone()
    R.mf_sgd_local(Ur, Ir, uid.cpu(), iid.cpu(), r.cpu(), 0.01)
    ops.mf_sgd_tiled(U, I, rec, ptr, 0, T, Rt, 0.01)
    # distinct users: item deltas are summed against the item's value at the chunk
    # start; a tile with > 4096 ratings runs in 2 chunks (second sees the first's sum)
    torch.testing.assert_close(I.cpu(), Ir, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(U.cpu(), Ur, rtol=1e-2, atol=2e-5)


def test_ring_known_and_known_list_sampling_match_reference():
    nu, ni, mem = 500, 3000, 8
    ring_g = torch.full((nu * mem,), -1, dtype=torch.int32, device=DEV)
    cur_g = torch.zeros(nu, dtype=torch.int32, device=DEV)
    ring_r, cur_r = ring_g.cpu().clone(), cur_g.cpu().clone()
    flag_g = torch.zeros(ni, dtype=torch.int32, device=DEV)
    lst_g = torch.zeros(ni, dtype=torch.int32, device=DEV)
    cnt_g = torch.zeros(1, dtype=torch.int32, device=DEV)
    for step in range(3):  # unique users per push: slot order is deterministic
        uid = torch.randperm(nu, dtype=torch.int32)[:400]
        iid = torch.randint(0, ni // 2, (400,), dtype=torch.int32)
        ops.ring_push(ring_g, cur_g, uid.to(DEV), iid.to(DEV), mem)
        R.ring_push(ring_r, cur_r, uid, iid, mem)
        ops.known_append(flag_g, lst_g, cnt_g, iid.to(DEV))
    assert torch.equal(ring_g.cpu(), ring_r) and torch.equal(cur_g.cpu(), cur_r)
    n_known = int(cnt_g[0])
    known_set = set(lst_g[:n_known].cpu().tolist())
    assert known_set == set(torch.nonzero(flag_g.cpu()).flatten().tolist()) and len(known_set) == n_known
    uid = torch.randint(0, nu, (1000,), dtype=torch.int32)
    pos = torch.randint(0, ni, (1000,), dtype=torch.int32)
    g = ops.sample_uniform_reject(1000, 3, ni, pos.to(DEV), uid.to(DEV), ring_g, mem, seed=4, counter=2,
                                  device=DEV, known=lst_g, known_count=cnt_g).cpu()
    r = R.sample_uniform_reject(1000, 3, ni, pos, uid, ring_r, mem, 4, 2, lst_g.cpu(), n_known)
    assert torch.equal(g, r)  # same known list on both sides
    assert set(g.tolist()) <= known_set


@pytest.mark.parametrize("phases", [1, 3])
@pytest.mark.parametrize("rec8", [False, True])
def test_mf_sgd_tiled_delta_mode_equals_in_place(phases, rec8):
    """The PS path's delta mode (item rows read-only, the summed deltas written to a
    separate buffer, later user phases accumulating) == the in-place kernel's row
    change.  Unique users (no Hogwild race); items repeat ~60x, so tiles span several
    LDS chunks and some tiles and rows get no ratings at all."""
    D, nu, ni, B = 64, 400_000, 6000, 200_000
    U0 = torch.rand(nu, D, device=DEV) * 0.1
    I0 = torch.rand(ni, D, device=DEV) * 0.1
    uid = torch.randperm(nu, device=DEV)[:B].to(torch.int32)
    iid = torch.randint(0, ni - 700, (B,), device=DEV, dtype=torch.int32)  # the last tiles stay empty
    iid[iid % 7 == 3] = 11  # a hot row: many chunks in its tile
    r = torch.rand(B, device=DEV)
    Rt = ops.tile_rows_for(D, ni, 1)
    T = -(-ni // Rt)
    upp = -(-nu // phases)
    part = ops.TilePartitioner(1, [ni], Rt, T, DEV, rec8=rec8, phases=phases, users_per_phase=upp)
    ptr, rec = part.run(uid, iid, r)
    assert int((ptr[1:T + 1] - ptr[:T]).max()) > 2 * 4608  # a multi-chunk tile
    U1, I1 = U0.clone(), I0.clone()
    lr = 1e-3  # the hot row sums ~28k ratings' deltas: a small step keeps it bounded
    for p in range(phases):
        ops.mf_sgd_tiled(U1, I1, rec, ptr, 2 * p, T, Rt, lr, 0.01)
    U2, I2 = U0.clone(), I0.clone()
    delta = torch.full_like(I2, float("nan"))  # every row must be written
    for p in range(phases):
        ops.mf_sgd_tiled(U2, I2, rec, ptr, 2 * p, T, Rt, lr, 0.01, delta=delta, delta_init=p == 0)
    torch.cuda.synchronize()
    assert torch.equal(I2, I0)  # read-only
    assert not torch.isnan(delta).any()
    assert torch.equal(delta[ni - 600:], torch.zeros_like(delta[ni - 600:]))
    torch.testing.assert_close(U2, U1, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(I0 + delta, I1, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,k", [(4096, 100), (4096, 128), (1000, 100), (300, 37)])
def test_topk_select_fresh_equals_block_merge(n, k):
    """``topk_merge(fresh=True)`` (one wave per row, ``fps_topk_select``) == the block
    merge into empty lists, bit for bit: distinct scores, ties at the k-th key broken by
    smaller id, and rows whose ties overflow the wave's sort (redone by the block kernel)."""
    g = torch.Generator(device=DEV).manual_seed(n + k)
    B = 777
    S = torch.randn(B, n, device=DEV, generator=g)
    S[1::5] = torch.round(S[1::5] * 4) / 4  # heavy ties, some at the k-th key
    # > 256 keys tied at the k-th key: the wave's sort cannot hold them, the block kernel
    # redoes those rows (within its own exact range, < 924 ties)
    a, t = k // 2, min(600, n - k // 2)
    S[2::9] = -torch.rand(S[2::9].shape, device=DEV, generator=g) - 2.0
    S[2::9, :a] = 5.0
    S[2::9, a:a + t] = 1.0
    S[3, : n // 2] = float("-inf")
    ids = torch.randperm(10 * n, device=DEV, generator=g)[:n]
    out = []
    for fresh in (True, False):
        bs = torch.full((B, k), float("-inf"), device=DEV)
        bi = torch.full((B, k), -1, dtype=torch.long, device=DEV)
        ops.topk_merge(S, ids, bs, bi, fresh=fresh)
        out.append((bs, bi))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])
    ref = torch.topk(S, k, dim=1).values
    assert torch.equal(out[0][0], ref)


def test_scalar_rows_gather_apply_large():
    """D = 1 (PA's weight vector): the scalar kernels (8 rows in flight per lane) over more
    rows than one workgroup covers, with repeats (atomic add) and -1 padding, vs torch."""
    g = torch.Generator(device=DEV).manual_seed(5)
    tab = torch.randn(200_003, 1, device=DEV, generator=g)
    idx = torch.randint(0, 200_003, (70_001,), device=DEV, dtype=torch.int32, generator=g)
    idx[::9] = -1
    out = ops.gather_rows(tab, idx)
    ref = torch.where((idx >= 0).view(-1, 1), tab[idx.long().clamp_min(0)], torch.zeros_like(out))
    assert torch.equal(out, ref)
    delta = torch.randn(idx.numel(), 1, device=DEV, generator=g)
    exp = tab.clone()
    ok = idx >= 0
    exp.index_add_(0, idx[ok].long(), delta[ok])
    ops.apply_rows(tab, idx, delta, "add")
    torch.testing.assert_close(tab, exp, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shape,dtype", [((1000,), torch.int32), ((777, 1), torch.float32), ((513, 300), torch.bfloat16),
                                         ((64, 7), torch.float32), ((90, 3), torch.bfloat16), ((50, 5), torch.uint8)])
def test_segment_fill_matches_torch(shape, dtype):
    """The emulated all-to-all's receive fill (``ops.segment_fill``): segment j = the first
    rows[j] rows of src, tiled past its end -- 16-B, 4-B, 2-B and 1-B word kernels against
    the torch loop on the CPU."""
    g = torch.Generator().manual_seed(shape[0])
    src = (torch.randint(0, 100, shape, generator=g).to(dtype) if dtype in (torch.int32, torch.uint8)
           else torch.randn(shape, generator=g).to(dtype))
    k = shape[0]
    rows = [k, 0, k // 3, 2 * k + 5, 1, k - 1, 3 * k]
    n = sum(rows)
    ref = torch.empty((n,) + shape[1:], dtype=dtype)
    ops.segment_fill(src, rows, ref)
    off = 0
    for m in rows:  # the definition, row by row
        for i in range(0, m, max(1, m // 7)):
            assert torch.equal(ref[off + i], src[i % k])
        off += m
    for min_us in (0.0, 50.0):  # the timed (link) launch runs on at most 256 workgroups
        out = torch.full((n + 3,) + shape[1:], 7, dtype=dtype, device=DEV)
        ops.segment_fill(src.to(DEV), rows, out, min_us=min_us)
        assert torch.equal(out[:n].cpu(), ref)
        assert bool((out[n:].cpu() == 7).all())  # nothing past the segments is written


def test_segment_fill_lasts_its_link_time():
    """``segment_fill(min_us=...)`` (the emulated link): the launch lasts at least the
    modelled transfer time, also with nothing to write, and still writes its rows."""
    src = torch.arange(4096, dtype=torch.float32, device=DEV).view(1024, 4)
    out = torch.zeros(2048, 4, device=DEV)
    for rows, want_us in (([1024, 1024], 1500.0), ([0], 800.0)):
        ops.segment_fill(src, rows, out, min_us=10.0)  # warm-up
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ops.segment_fill(src, rows, out, min_us=want_us)
        b.record()
        torch.cuda.synchronize()
        assert a.elapsed_time(b) * 1e3 >= 0.95 * want_us
    assert torch.equal(out, torch.cat([src, src]))


def test_pack_counts_kernel_matches_cpu():
    c = torch.randint(0, 1 << 20, (300,), dtype=torch.int32)
    for request, flag in ((False, 0), (True, 1), (True, 0)):
        got = ops.pack_counts(c.to(DEV), 300, request, flag).cpu()
        assert torch.equal(got, ops.pack_counts(c, 300, request, flag))
