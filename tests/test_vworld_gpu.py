"""GPU: the N > 1 paths under the stream-faithful virtual world (``parallel/vworld.py``).

N rank threads share cuda:0, each on its own compute stream; every transfer runs
on a link stream after both sides posted, behind an injected xGMI-like delay, and
``Work.wait()`` is a stream wait -- RCCL's contract, not gloo's host-synchronous
one.  The async results must equal the host-synchronous reference (``mode="sync"``)
BIT FOR BIT where the kernels are deterministic (rotation and PS-path MF with
distinct users and items inside each micro-batch), and to fp32 summation order
where they use float atomics (PA request plans, SGNS).  The mutation tests remove
one ``w.wait()`` from ``parallel/rotation.py`` and check the harness sees the race.
"""
import importlib.util
import os
import sys

import pytest
import torch

from flink_parameter_server_1_amd.parallel import vworld
from flink_parameter_server_1_amd.parallel.vworld import run_virtual

pytestmark = pytest.mark.gpu

NU, NI, D, B, STEPS = 40_000, 6_000, 64, 3_000, 4


def _unique_batches(rank, world, steps, nu_local, ni, b, seed=7):
    """Per step: ``b`` distinct local users and ``b`` distinct items (no Hogwild
    collision, one rating per item row: the tiled kernel is then deterministic)."""
    g = torch.Generator(device="cpu").manual_seed(seed * 7919 + rank)
    out = []
    for _ in range(steps):
        u = torch.randperm(nu_local, generator=g)[:b].to(torch.int32)
        i = torch.randperm(ni, generator=g)[:b].to(torch.int32)
        r = torch.rand(b, generator=g)
        out.append((u.cuda(), i.cuda(), r.cuda()))
    return out


def _mf_run(comm, exchange, schedule, steps=STEPS, batch=B, rotation_cls=None, overlap=True):
    from flink_parameter_server_1_amd.models.mf import fast

    cfg = fast.MFConfig(num_users=NU, num_items=NI, dim=D, learning_rate=0.05, range_min=0.0, range_max=0.2,
                        exchange=exchange, rotation=schedule, overlap_substeps=overlap)
    m = fast.DistributedMF(cfg, comm)
    if rotation_cls is not None:  # the mutant rotation (same schedule, one wait removed)
        m.rot = rotation_cls(comm, m.items.weight, NI, schedule)
    assert m.sgd_mode == "tiled"
    for u, i, r in _unique_batches(comm.rank, comm.world, steps, m.users.n_local, NI, batch):
        m.step(u, i, r)
    m.flush()
    ids, vals = m.item_vectors(only_touched=True)
    wait = m.rot.wait_ms() if exchange == "rotate" else 0.0
    return ids.cpu(), vals.cpu(), m.U.cpu().clone(), wait


def _assert_same(a, b, exact=True):
    for ra, rb in zip(a, b):
        assert torch.equal(ra[0], rb[0])
        if exact:
            assert torch.equal(ra[1], rb[1]), (ra[1] - rb[1]).abs().max()
            assert torch.equal(ra[2], rb[2]), (ra[2] - rb[2]).abs().max()
        else:
            torch.testing.assert_close(ra[1], rb[1], rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(ra[2], rb[2], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("schedule", ["bidir", "ring"])
def test_rotation_async_equals_sync_bitwise(world, schedule):
    sync = run_virtual(_mf_run, world, "rotate", schedule, mode="sync")
    # ~1 ms per block transfer: far longer than a sub-step's compute at this size,
    # so any read of a block before its wait, or reuse of a buffer before its send
    # completed, reads the wrong rows
    res, vw = run_virtual(_mf_run, world, "rotate", schedule, mode="async", latency_us=1000.0,
                          return_world=True)
    _assert_same(res, sync)
    assert vw.transfers > 0 and sum(vw.link_us.values()) > 0
    # the compute streams really waited for the (slow) transfers
    assert all(r[3] > 0.5 for r in res), [r[3] for r in res]


def test_rotation_sync_equals_sequential_reference():
    """The host-synchronous virtual world runs the schedule of tests/test_rotation.py's
    single-process sequential replay (CPU fp32 reference, fp32 rounding apart)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from flink_parameter_server_1_amd.ops import reference as R

    world = 4
    res = run_virtual(_mf_run, world, "rotate", "bidir", mode="sync")
    # sequential replay: rank by rank per sub-step is equivalent to rank by rank per
    # micro-batch here (every rank's users are disjoint and every item appears in
    # ONE batch of ONE rank per step at most once ... across ranks items repeat, so
    # the replay walks the rotation schedule)
    from flink_parameter_server_1_amd.models.mf.fast import MFConfig
    from flink_parameter_server_1_amd.parallel.rotation import block_rows, layout_world, shard_halves
    from flink_parameter_server_1_amd.parallel.table import ShardedTable

    cfg = MFConfig(num_users=NU, num_items=NI, dim=D, learning_rate=0.05, range_min=0.0, range_max=0.2)
    init = ("uniform", cfg.range_min, cfg.range_max)
    users = [ShardedTable(NU, D, r, world, "hash", init, cfg.user_seed(), track_touched=False).weight
             for r in range(world)]
    items = ShardedTable(NI, D, 0, 1, "hash", init, cfg.item_seed(), track_touched=False).weight
    Wv = layout_world(world, "bidir")
    half = torch.tensor(shard_halves(NI, Wv))
    data = [[tuple(x.cpu() for x in t) for t in _unique_batches(r, world, STEPS, users[r].shape[0], NI, B)]
            for r in range(world)]
    K = 2 * world
    for s in range(STEPS):
        for t in range(K):
            for r in range(world):
                u, i, rt = data[r][s]
                blk, _ = R.rot_block_of(i, Wv, half)
                mine = [(2 * r + t) % K, K + (2 * r + 1 - t) % K]
                sel = (blk == mine[0]) | (blk == mine[1])
                R.mf_sgd_local(users[r], items, u[sel], i[sel], rt[sel], cfg.learning_rate)
    ids = torch.cat([x[0] for x in res])
    vals = torch.cat([x[1] for x in res])
    torch.testing.assert_close(vals, items[ids.long()], rtol=1e-5, atol=1e-6)
    for r in range(world):
        torch.testing.assert_close(res[r][2], users[r], rtol=1e-5, atol=1e-6)


def _load_mutant(line: str, count: int = 1):
    """``parallel/rotation.py`` with ``line`` (a ``w.wait()`` of a given indentation)
    replaced by ``pass``: a real source mutation, loaded as its own module."""
    from flink_parameter_server_1_amd.parallel import rotation

    src = open(rotation.__file__).read()
    line = "\n" + line  # the whole line, at exactly this indentation
    assert src.count(line) == count, (line, src.count(line))
    mutated = src.replace(line, line.replace("w.wait()", "pass"), count)
    spec = importlib.util.spec_from_loader("fps_rotation_mutant", loader=None)
    mod = importlib.util.module_from_spec(spec)
    mod.__dict__["__package__"] = "flink_parameter_server_1_amd.parallel"
    exec(compile(mutated, rotation.__file__ + " (mutant)", "exec"), mod.__dict__)
    return mod


@pytest.mark.parametrize("schedule", ["bidir", "ring"])
def test_mutation_missing_substep_wait_is_detected(schedule):
    """Remove the ``w.wait()`` of ``RingRotation.end`` (the compute of the next
    sub-step no longer waits for the block it reads): the async world must produce
    different numbers; the sync world (gloo's semantics) cannot see the bug."""
    # sub-steps on one stream: with alternating streams (the default) the same wait is
    # also issued for the posting stream, and the virtual world's waits block the host
    # until the delayed copy is issued (a host-timed link cannot hand out its event
    # earlier) -- the host would then launch the next sub-step after the copy anyway
    mutant = _load_mutant("                w.wait()\n")
    world = 4
    good = run_virtual(_mf_run, world, "rotate", schedule, mode="sync", overlap=False)
    hidden = run_virtual(_mf_run, world, "rotate", schedule, mode="sync", rotation_cls=mutant.RingRotation,
                         overlap=False)
    _assert_same(hidden, good)  # a host-synchronous transport hides the race
    bad = run_virtual(_mf_run, world, "rotate", schedule, mode="async", latency_us=1000.0,
                      rotation_cls=mutant.RingRotation, overlap=False)
    differs = any(not torch.equal(b[1], g[1]) or not torch.equal(b[2], g[2]) for b, g in zip(bad, good))
    assert differs, "the virtual world did not expose the missing wait"


def test_mutation_missing_home_wait_is_detected():
    """Remove the wait of ``RingRotation.home``: blocks are copied home before they arrive."""
    mutant = _load_mutant("            w.wait()\n")
    world = 2
    good = run_virtual(_mf_run, world, "rotate", "bidir", mode="sync")
    bad = run_virtual(_mf_run, world, "rotate", "bidir", mode="async", latency_us=1000.0,
                      rotation_cls=mutant.RingRotation)
    assert any(not torch.equal(b[1], g[1]) for b, g in zip(bad, good))


@pytest.mark.parametrize("world", [2, 4])
def test_mf_ps_path_async_equals_sync_bitwise(world):
    """The reference's pull / push protocol (``exchange="ps"``: dedup, count exchange,
    key / row / delta all-to-alls, staleness-1 pipeline) under RCCL semantics."""
    sync = run_virtual(_mf_run, world, "ps", "bidir", mode="sync")
    res = run_virtual(_mf_run, world, "ps", "bidir", mode="async", latency_us=300.0)
    _assert_same(res, sync)


def _pa_run(comm, dedup, capacity=None):
    from flink_parameter_server_1_amd.models.pa.fast import DistributedPA, PAConfig, synthetic_sparse_batch

    F = 1 << 22
    m = DistributedPA(PAConfig(feature_count=F, kind="binary", local_direct=False, capacity=capacity), comm)
    assert m.ps.fixed() == (capacity is not None)
    m.ps.dedup_mode = dedup
    for s in range(6):
        m.train_step(*synthetic_sparse_batch(2048, 32, F, seed=comm.rank + 3, step=s % 3, device="cuda"))
    ids, w = m.dump()
    o = torch.argsort(ids)
    return ids[o].cpu(), w[o].reshape(-1).cpu()


@pytest.mark.parametrize("dedup", [True, False])
def test_pa_ps_path_async_equals_sync(dedup):
    sync = run_virtual(_pa_run, 4, dedup, mode="sync")
    res = run_virtual(_pa_run, 4, dedup, mode="async", latency_us=300.0)
    for (ia, wa), (ib, wb) in zip(res, sync):
        assert torch.equal(ia, ib)
        torch.testing.assert_close(wa, wb, rtol=1e-4, atol=1e-6)  # float atomics: summation order only


@pytest.mark.parametrize("dedup", [True, False])
def test_pa_fixed_shape_plans_async_equals_sync_and_dynamic(dedup):
    """Fixed-shape plans (``TensorPS.capacity``: one [W, C + 2] key all-to-all, padded
    row / delta all-to-alls, nothing read on the host) under RCCL semantics: async ==
    sync, and both == the dynamic plans' model (float atomics: summation order)."""
    cap = 2048 * 32
    sync = run_virtual(_pa_run, 4, dedup, cap, mode="sync")
    res = run_virtual(_pa_run, 4, dedup, cap, mode="async", latency_us=300.0)
    dyn = run_virtual(_pa_run, 4, dedup, mode="sync")
    for (ia, wa), (ib, wb), (ic, wc) in zip(res, sync, dyn):
        assert torch.equal(ia, ib) and torch.equal(ia, ic)
        torch.testing.assert_close(wa, wb, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(wa, wc, rtol=1e-4, atol=1e-6)


def test_virtual_world_reports_collective_desync():
    def bad(comm):
        x = torch.ones(4, device="cuda")
        if comm.rank == 0:
            comm.all_reduce(x)
        else:
            comm.all_gather(x)

    with pytest.raises(vworld.VirtualWorldAborted, match="desync"):
        run_virtual(bad, 2, timeout_s=20)


def _sgns_run(comm):
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus

    m = DistributedSGNS(SGNSConfig(vocab_size=50_000, dim=128, window=4, learning_rate=0.01), comm=comm)
    toks = synthetic_corpus(200_000, 50_000, seed=comm.rank, device="cuda")
    c, o = skipgram_pairs(toks, 4, torch.Generator(device="cuda").manual_seed(comm.rank))
    P = 8192
    for i in range(8):
        m.step(c[i * P:(i + 1) * P], o[i * P:(i + 1) * P])
    m.flush()
    ids, w = m.embeddings()
    o_ = torch.argsort(ids)
    return ids[o_].cpu(), w[o_].cpu(), m.ps_in.stats["host_stalls"] + m.ps_out.stats["host_stalls"]


def test_sgns_pipeline_async_equals_sync():
    """SGNS through the two-table one-step-ahead planner (one count exchange per
    micro-batch) under RCCL semantics; its kernels sum with float atomics."""
    sync = run_virtual(_sgns_run, 4, mode="sync")
    res = run_virtual(_sgns_run, 4, mode="async", latency_us=300.0)
    for a, b in zip(res, sync):
        assert torch.equal(a[0], b[0])
        torch.testing.assert_close(a[1], b[1], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("schedule", ["bidir", "ring"])
def test_emulated_links_model_transfers_without_changing_results(schedule):
    """``EmulatedRotation(link_gbps=...)`` (rank 0's schedule with rank-symmetric
    host-timed links): the modelled transfers never touch the blocks (results equal
    the link-free emulation bit for bit); a fast link hides behind the sub-steps,
    a 0.2 GB/s one (~0.48 ms per 96 KB quarter-shard block, far longer than a
    sub-step of 375 ratings) makes the compute stream wait, and the wait is reported."""
    from flink_parameter_server_1_amd.models.mf import fast

    out = {}
    for gbps in (0.0, 50.0, 0.2):
        cfg = fast.MFConfig(num_users=NU, num_items=NI, dim=D, learning_rate=0.05, range_min=0.0, range_max=0.2,
                            exchange="rotate", rotation=schedule, emulate_world=4, emulate_link_gbps=gbps)
        m = fast.DistributedMF(cfg)
        for u, i, r in _unique_batches(0, 4, 3, m.users.n_local, NI, B):
            m.step(u, i, r)
        m.flush()
        torch.cuda.synchronize()
        out[gbps] = (m.I.cpu().clone(), m.U.cpu().clone(), m.rot.wait_ms(), m.rot.bytes_sent)
        m.rot.close()
    assert torch.equal(out[0.0][0], out[50.0][0]) and torch.equal(out[0.0][1], out[50.0][1])
    assert torch.equal(out[0.0][0], out[0.2][0]) and torch.equal(out[0.0][1], out[0.2][1])
    assert out[0.0][2] == 0.0 and out[0.0][3] == 0
    assert out[50.0][3] > 0
    subs = 3 * (8 - 1)  # transfers per step: every sub-step but the first
    assert out[0.2][2] > 0.25 * subs  # ms: most of the ~0.48 ms per transfer is exposed
    assert out[50.0][2] < out[0.2][2] / 4


def _mf_topk_run(comm, capacity):
    from flink_parameter_server_1_amd.models.mf.topk_tensor import (as_reference_records,
                                                                    ps_online_learner_and_generator_tensor)
    from flink_parameter_server_1_amd.core.messages import Right

    users, items, B = 2000, 4096, 256
    g = torch.Generator(device="cpu").manual_seed(21)  # the same broadcast input on every rank
    batches = [(torch.randint(0, users, (B,), generator=g), torch.randperm(items, generator=g)[:B],
                torch.arange(s * B, (s + 1) * B), torch.rand(B, generator=g)) for s in range(6)]
    out = ps_online_learner_and_generator_tensor(batches, users, items, num_factors=16, learning_rate=0.05, K=10,
                                                 worker_k=10, user_memory=4, bucket_size=256, seed=3, comm=comm,
                                                 capacity=capacity, range_min=-0.1, range_max=0.1)
    recs = as_reference_records(out)
    ps_users = {}
    for e in out:
        if isinstance(e, Right):
            ids, vals = e.value
            for k, v in zip(ids.tolist(), vals.tolist()):
                ps_users[k] = v
    return recs, ps_users


@pytest.mark.parametrize("capacity", [None, 256])
def test_mf_topk_async_equals_sync(capacity):
    """Online MF + top-K at N = 2 under RCCL semantics (candidate all-gather, PS pull /
    push, fixed-shape plans with ``capacity``): rank 0's top-K lists and every rank's PS
    user vectors equal the host-synchronous world's (distinct items per batch: no
    float-atomic races on the items; repeated users' deltas sum in fp32 atomics order)."""
    sync = run_virtual(_mf_topk_run, 2, capacity, mode="sync")
    res = run_virtual(_mf_topk_run, 2, capacity, mode="async", latency_us=200.0)
    assert len(res[0][0]) == 6 * 256 and res[1][0] == []
    for (ra, ua), (rb, ub) in zip(res, sync):
        assert [r[:3] for r in ra] == [r[:3] for r in rb]
        for a, b in zip(ra, rb):
            assert [x[1] for x in a[3]] == [x[1] for x in b[3]]
            assert [x[0] for x in a[3]] == [x[0] for x in b[3]]
        assert ua.keys() == ub.keys()  # user deltas of repeated users sum with atomics: fp32 order only
        for k in ua:
            torch.testing.assert_close(torch.tensor(ua[k]), torch.tensor(ub[k]), rtol=1e-5, atol=1e-6)
