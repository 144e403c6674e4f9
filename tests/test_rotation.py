"""Item-block ring rotation (stratified MF-SGD over the ring) on gloo, W = 2..4."""
import pytest
import torch

from dist_utils import run_ranks
from flink_parameter_server_1_amd.ops import reference as R
from flink_parameter_server_1_amd.parallel.rotation import block_rows, shard_halves

NU, NI, D, B, STEPS = 700, 301, 8, 500, 3


def test_block_layout_covers_every_item_once():
    for W in (1, 2, 3, 5, 8):
        half = torch.tensor(shard_halves(NI, W))
        rows = block_rows(NI, W)
        b, row = R.rot_block_of(torch.arange(NI), W, half)
        assert sum(rows) == NI
        for k in range(2 * W):
            sel = row[b == k]
            assert sorted(sel.tolist()) == list(range(rows[k]))


def test_rot_partition_reference_groups_by_block():
    W = 3
    half = torch.tensor(shard_halves(NI, W))
    uid = torch.randint(0, 50, (400,), dtype=torch.int32)
    iid = torch.randint(0, NI, (400,), dtype=torch.int32)
    r = torch.rand(400)
    counts, ptr, u, row, rr = R.rot_partition(uid, iid, r, W, half)
    b, rowg = R.rot_block_of(iid, W, half)
    for k in range(2 * W):
        a, e = int(ptr[k]), int(ptr[k + 1])
        m = b == k
        assert torch.equal(u[a:e], uid[m]) and torch.equal(row[a:e], rowg[m].int()) and torch.equal(rr[a:e], r[m])


def _rot_train(rank, world, steps, dim=D, phases=0, schedule="bidir"):
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm()
    cfg = MFConfig(num_users=NU, num_items=NI, dim=dim, learning_rate=0.1, range_min=0.0, range_max=0.3,
                   user_phases=phases, rotation=schedule)
    m = DistributedMF(cfg, comm)
    assert m.sgd_mode != "tiled" or m.user_phases == max(phases, 1)
    assert m.exchange == "rotate"
    assert m.sgd_mode == ("tiled" if dim in (16, 32, 64) else "flat")
    data = SyntheticRatings(NU, NI, B * steps, rank, world, seed=3)
    for s in range(steps):
        m.step(*data.batch(s, B))
    se = m.sq_err(*data.batch(0, B))  # flushes: blocks return home
    assert m.rot.at_rest
    ids, vals = m.item_vectors(only_touched=True)
    uids, uv = m.user_vectors()
    return ids, vals, uids, uv.clone(), se, m.rot.bytes_sent


def _blocks_of(schedule, world, r, t):
    """Partition-layout blocks rank r updates in sub-step t."""
    K = 2 * world
    if schedule == "ring":
        return [(2 * r + t) % K]
    return [(2 * r + t) % K, K + (2 * r + 1 - t) % K]


def _emulate(world, steps, dim=D, phases=0, schedule="bidir"):
    """Single-process replay of the same schedule (sub-step t: rank r on its blocks
    of ``_blocks_of``, one after the other, phases outermost)."""
    from flink_parameter_server_1_amd import ops
    from flink_parameter_server_1_amd.models.mf.fast import MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.rotation import layout_world
    from flink_parameter_server_1_amd.parallel.table import ShardedTable

    cfg = MFConfig(num_users=NU, num_items=NI, dim=dim, learning_rate=0.1, range_min=0.0, range_max=0.3)
    init = ("uniform", cfg.range_min, cfg.range_max)
    users = [ShardedTable(NU, dim, r, world, "hash", init, cfg.user_seed(), track_touched=False) for r in range(world)]
    items = ShardedTable(NI, dim, 0, 1, "hash", init, cfg.item_seed(), track_touched=False).weight
    Wv = layout_world(world, schedule)
    tiled = dim in ops.TILED_DIMS
    if tiled:  # same tile geometry as DistributedMF
        rows_max = max(block_rows(NI, Wv))
        Rt = ops.tile_rows_for(dim, rows_max, Wv)
        Tt = -(-rows_max // Rt)
    half = torch.tensor(shard_halves(NI, Wv))
    data = [SyntheticRatings(NU, NI, B * steps, r, world, seed=3) for r in range(world)]
    K = 2 * world
    KB = 2 * Wv  # blocks per phase in the partition layout
    P = max(phases, 1) if tiled else 1
    seen = torch.zeros(NI, dtype=torch.bool)
    for s in range(steps):
        parts = []
        for r in range(world):
            uid, iid, rating = data[r].batch(s, B)
            seen[iid.long()] = True
            if tiled:
                upp = -(-users[r].n_local // P)  # user phases as DistributedMF cuts them
                ptr, u_, row_, r_ = R.tile_partition(uid, iid, rating, Wv, half, Rt, Tt, P, upp)
                # (phase p, block b)'s segment: ptr[(p*KB + b)*T] .. ptr[(p*KB + b + 1)*T]
                parts.append((None, ptr[:: Tt], u_, row_, r_))
            else:
                parts.append(R.rot_partition(uid, iid, rating, Wv, half))
        for t in range(K):
            for r in range(world):
                _, ptr, u, row, rr = parts[r]
                blks = {}
                for b in _blocks_of(schedule, world, r, t):
                    q, h = b // 2, b % 2
                    n_local = (NI - q + Wv - 1) // Wv
                    lo = 0 if h == 0 else int(half[q])
                    hi = int(half[q]) if h == 0 else n_local
                    gid = q + Wv * torch.arange(lo, hi)
                    blks[b] = (gid, items[gid].clone())
                for p in range(P):  # the phases of a sub-step run in order on the resident blocks
                    for b, (gid, blk) in blks.items():
                        a, e = int(ptr[p * KB + b]), int(ptr[p * KB + b + 1])
                        # user rows: last writer (user_update "auto" = "store" at every world size)
                        R.mf_sgd_local(users[r].weight, blk, u[a:e], row[a:e], rr[a:e], cfg.learning_rate,
                                       user_atomic=False)
                for b, (gid, blk) in blks.items():
                    items[gid] = blk
    return users, items, seen


@pytest.mark.parametrize("schedule", ["bidir", "ring"])
@pytest.mark.parametrize("world,dim,phases", [(2, D, 0), (3, D, 0), (4, D, 0), (2, 16, 0), (3, 32, 0), (2, 16, 3),
                                              (3, 32, 2)])
def test_rotation_equals_sequential_schedule(world, dim, phases, schedule):
    res = run_ranks(_rot_train, world, STEPS, dim, phases, schedule)
    # single thread like the ranks: index_put with duplicate users is last-writer-wins,
    # and which write is last depends on the thread split
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        users, items, seen = _emulate(world, STEPS, dim, phases, schedule)
    finally:
        torch.set_num_threads(nt)
    ids = torch.cat([x[0] for x in res])
    vals = torch.cat([x[1] for x in res])
    # dump covers exactly the rated items
    assert torch.equal(torch.sort(ids).values, torch.nonzero(seen).flatten())
    torch.testing.assert_close(vals, items[ids], rtol=1e-6, atol=1e-7)
    for r in range(world):
        torch.testing.assert_close(res[r][3], users[r].weight, rtol=1e-6, atol=1e-7)
    # every sub-step after the first moved blocks on every rank
    assert all(x[5] > 0 for x in res)


def test_bidir_moves_half_the_bytes_per_link_direction():
    """Per sub-step a bidir rank sends two quarter-shard blocks to two different
    neighbours (at W > 2), the single ring one half-shard block to one: the same
    total bytes, split over two link directions."""
    world = 4
    bidir = run_ranks(_rot_train, world, 1, D, 0, "bidir")
    ring = run_ranks(_rot_train, world, 1, D, 0, "ring")
    for b, g in zip(bidir, ring):
        assert abs(b[5] - g[5]) <= 0.02 * g[5]


def _rot_vs_ps(rank, world, exchange):
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm()
    cfg = MFConfig(num_users=600, num_items=300, dim=8, learning_rate=0.2, range_min=0.0, range_max=0.3,
                   exchange=exchange)
    m = DistributedMF(cfg, comm)
    data = SyntheticRatings(600, 300, 20000, rank, world, seed=11, truth_dim=4)
    first = m.rmse(*data.batch(0, 4000))
    for s in range(25):
        m.step(*data.batch(s % 5, 4000))
    return first, m.rmse(*data.batch(0, 4000))


def test_rotation_learns_like_ps_path():
    rot = run_ranks(_rot_vs_ps, 2, "rotate")
    ps = run_ranks(_rot_vs_ps, 2, "ps")
    assert rot[0][1] < 0.6 * rot[0][0]
    assert rot[0][1] < 1.2 * ps[0][1]


def test_rotation_single_rank_matches_local_block_order():
    """W = 1 rotate: the two half-blocks alternate in place; equals the emulation."""
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings

    cfg = MFConfig(num_users=NU, num_items=NI, dim=D, learning_rate=0.1, range_min=0.0, range_max=0.3,
                   exchange="rotate", rotation="ring")
    m = DistributedMF(cfg)
    data = SyntheticRatings(NU, NI, B * STEPS, 0, 1, seed=3)
    for s in range(STEPS):
        m.step(*data.batch(s, B))
    m.flush()
    users, items, _ = _emulate(1, STEPS, schedule="ring")
    torch.testing.assert_close(m.I, items, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(m.U, users[0].weight, rtol=1e-6, atol=1e-7)


def test_emulated_world_runs_rank0_schedule():
    """emulate_world = N on one process: rank 0's users (1/N of them), the
    N-rank block layout, and exactly _blocks_of(r=0) per sub-step."""
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings

    for schedule in ("bidir", "ring"):
        cfg = MFConfig(num_users=NU, num_items=NI, dim=D, learning_rate=0.1, range_min=0.0, range_max=0.3,
                       exchange="rotate", rotation=schedule, emulate_world=4)
        m = DistributedMF(cfg)
        assert m.users.n_local == (NU + 3) // 4 and m.rot.K == 8
        m.rot.begin()
        for t in range(8):
            assert [g for g, _ in m.rot.active_blocks()] == _blocks_of(schedule, 4, 0, t)
            m.rot.end()
        m.rot.home()
        I0 = m.I.clone()
        data = SyntheticRatings(NU, NI, B * 2, 0, 4, seed=3)
        m.step(*data.batch(0, B))
        m.flush()
        assert not torch.equal(I0, m.I) and m.rot.at_rest
