"""GPU: the N > 1 paths on REAL ranks -- one process per GPU over RCCL (``nccl``) when
the box has >= 2 GPUs -- and, on every GPU box, the same bodies in the stream-faithful
virtual world (``parallel/vworld.py``: N rank threads on cuda:0 with RCCL's stream
contract and delayed links).

Each body runs on the world under test and is compared with a reference that cannot
share its bugs:

* the MF rotation and the MF PS path: the sequential fp32 CPU replay of
  ``parallel/verify.py`` (distinct users / items per batch: to fp32 rounding);
* PA (dynamic and fixed-shape plans), SGNS, online MF + top-K: the same body on the
  host-synchronous virtual world (gloo's semantics), float atomics to summation order;
* checkpoints: shards saved by N ranks, restored by N / 2 ranks (re-shard), dump equal.

``N = min(torch.cuda.device_count(), 8)``: the nccl cases skip below 2 GPUs (spawned
children are fresh interpreters; the parent only counts devices).  The reference
worker logic is ``FlinkParameterServer.scala:265-317,331-335`` (the worker <-> PS
shuffle and its feedback edge).
"""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dist_utils import run_nccl  # noqa: E402
from flink_parameter_server_1_amd.parallel.vworld import run_virtual  # noqa: E402

pytestmark = pytest.mark.gpu

N_GPUS = min(torch.cuda.device_count(), 8) if torch.cuda.is_available() else 0
BACKENDS = ["virtual", pytest.param("nccl", marks=pytest.mark.skipif(N_GPUS < 2, reason="needs >= 2 GPUs"))]


def _world(backend: str) -> int:
    return N_GPUS if backend == "nccl" else 4


def _run(backend, fn, world, *args):
    if backend == "nccl":
        return run_nccl(fn, world, *args)
    return run_virtual(fn, world, *args, mode="async", latency_us=300.0)


# ------------------------------------------------------------------ bodies (fn(comm, ...))
def _verify(comm, exchange, schedule, overlap):
    from flink_parameter_server_1_amd.parallel.verify import rotation_check

    return rotation_check(comm, schedule=schedule, exchange=exchange, overlap=overlap)


def _pa(comm, dedup, capacity):
    from flink_parameter_server_1_amd.models.pa.fast import DistributedPA, PAConfig, synthetic_sparse_batch

    F = 1 << 22
    m = DistributedPA(PAConfig(feature_count=F, kind="binary", local_direct=False, capacity=capacity), comm)
    m.ps.dedup_mode = dedup
    for s in range(6):
        m.train_step(*synthetic_sparse_batch(2048, 32, F, seed=comm.rank + 3, step=s % 3, device=comm.device))
    ids, w = m.dump()
    o = torch.argsort(ids)
    return ids[o].cpu(), w[o].reshape(-1).cpu()


def _sgns(comm):
    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus

    m = DistributedSGNS(SGNSConfig(vocab_size=50_000, dim=128, window=4, learning_rate=0.01), comm=comm)
    toks = synthetic_corpus(200_000, 50_000, seed=comm.rank, device=comm.device)
    c, o = skipgram_pairs(toks, 4, torch.Generator(device=comm.device).manual_seed(comm.rank))
    P = 8192
    for i in range(8):
        m.step(c[i * P:(i + 1) * P], o[i * P:(i + 1) * P])
    m.flush()
    ids, w = m.embeddings()
    o_ = torch.argsort(ids)
    return ids[o_].cpu(), w[o_].cpu()


def _mf_topk(comm, capacity):
    from flink_parameter_server_1_amd.core.messages import Right
    from flink_parameter_server_1_amd.models.mf.topk_tensor import (as_reference_records,
                                                                    ps_online_learner_and_generator_tensor)

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


def _pa_save(comm, directory):
    from flink_parameter_server_1_amd.models.pa.fast import DistributedPA, PAConfig, synthetic_sparse_batch
    from flink_parameter_server_1_amd.utils.io import save_table

    F = 1 << 20
    m = DistributedPA(PAConfig(feature_count=F, kind="binary", local_direct=False), comm)
    for s in range(4):
        m.train_step(*synthetic_sparse_batch(1024, 16, F, seed=comm.rank + 5, step=s, device=comm.device))
    save_table(m.table, os.path.join(directory, f"pa.shard{comm.rank}-of-{comm.world}.bin"), step=4)
    ids, w = m.dump()
    o = torch.argsort(ids)
    return ids[o].cpu(), w[o].reshape(-1).cpu()


def _pa_restore(comm, directory):
    from flink_parameter_server_1_amd.models.pa.fast import DistributedPA, PAConfig
    from flink_parameter_server_1_amd.utils.io import restore_table

    F = 1 << 20
    m = DistributedPA(PAConfig(feature_count=F, kind="binary", local_direct=False), comm)
    restore_table(m.table, os.path.join(directory, "pa.shard*-of-*.bin"))
    ids, w = m.dump()
    o = torch.argsort(ids)
    return ids[o].cpu(), w[o].reshape(-1).cpu()


def _pair_emb(comm, optimizer):
    """Config #5 scaled down: the range-sharded pair-embedding table under bounded
    staleness 2 (pushes of up to two later micro-batches in flight before a pull)."""
    from flink_parameter_server_1_amd.models.emb import DistributedPairEmbedding, PairEmbeddingConfig, \
        synthetic_pairs

    cfg = PairEmbeddingConfig(num_ids=2_000_000, dim=64, staleness=2, optimizer=optimizer, learning_rate=0.05)
    m = DistributedPairEmbedding(cfg, comm)
    batches = [synthetic_pairs(cfg.num_ids, 1 << 14, seed=comm.rank + 1, step=s, device=comm.device, zipf=3.0)
               for s in range(4)]
    loss0 = m.mean_loss(*batches[0])
    for s in range(12):
        m.step(*batches[s % 4])
    m.flush()
    loss1 = m.mean_loss(*batches[0])
    return m.table.weight.cpu().clone(), loss0, loss1, m.rows_pushed


def _model_load_wp(comm, wp, pp, capacity):
    from test_tensor_engine import _model_load

    return _model_load(comm.rank, comm.world, 50, 0, None, capacity, wp, pp, comm=comm)


# ------------------------------------------------------------------ tests
@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("capacity", [None, 7])
def test_model_load_worker_4_ps_3_exact(backend, capacity):
    """FlinkSimpleStackTest's model-load job (workerParallelism 4, psParallelism 3:
    FlinkSimpleStackTest.scala:135-138) on four ranks: shard ``|id| % 3`` on ranks 0-2,
    rank 3 has no shard -- the dump is exactly ``10 i + 3``."""
    W = 4 if backend == "virtual" else min(N_GPUS, 4)
    if W < 4:
        pytest.skip("needs 4 GPUs")
    res = _run(backend, _model_load_wp, W, 4, 3, capacity)
    dump = {}
    for r in res:
        for ids, vals in r:
            for k, v in zip(ids.tolist(), vals.reshape(-1).tolist()):
                assert k not in dump
                dump[k] = v
    assert dump == {k: 10.0 * k + 3 for k in range(50)}



@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("exchange,schedule,overlap", [("rotate", "bidir", "auto"), ("rotate", "ring", False),
                                                       ("rotate", "bidir", True), ("ps", "bidir", "auto")])
def test_mf_step_equals_sequential_replay(backend, exchange, schedule, overlap):
    res = _run(backend, _verify, _world(backend), exchange, schedule, overlap)
    assert all(r["verify_ok"] for r in res), res[0]
    assert res[0]["verify_world"] == _world(backend) and res[0]["verify_sgd_mode"] == "tiled"


@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("dedup,capacity", [(True, None), (False, None), (True, 2048 * 32)])
def test_pa_equals_host_synchronous_world(backend, dedup, capacity):
    W = _world(backend)
    res = _run(backend, _pa, W, dedup, capacity)
    ref = run_virtual(_pa, W, dedup, capacity, mode="sync")
    for (ia, wa), (ib, wb) in zip(res, ref):
        assert torch.equal(ia, ib)
        torch.testing.assert_close(wa, wb, rtol=1e-4, atol=1e-6)  # float atomics: summation order only


@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", BACKENDS)
def test_sgns_equals_host_synchronous_world(backend):
    W = _world(backend)
    res = _run(backend, _sgns, W)
    ref = run_virtual(_sgns, W, mode="sync")
    for a, b in zip(res, ref):
        assert torch.equal(a[0], b[0])
        torch.testing.assert_close(a[1], b[1], rtol=1e-4, atol=1e-6)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("capacity", [None, 256])
def test_mf_topk_equals_host_synchronous_world(backend, capacity):
    W = min(_world(backend), 4)
    res = _run(backend, _mf_topk, W, capacity)
    ref = run_virtual(_mf_topk, W, capacity, mode="sync")
    assert len(res[0][0]) == 6 * 256 and all(r[0] == [] for r in res[1:])
    for (ra, ua), (rb, ub) in zip(res, ref):
        assert [r[:3] for r in ra] == [r[:3] for r in rb]
        for a, b in zip(ra, rb):
            assert [x[1] for x in a[3]] == [x[1] for x in b[3]]
        assert ua.keys() == ub.keys()
        for k in ua:
            torch.testing.assert_close(torch.tensor(ua[k]), torch.tensor(ub[k]), rtol=1e-5, atol=1e-6)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", BACKENDS)
def test_checkpoint_saved_at_n_restores_at_half(backend, tmp_path):
    """Shards written by N ranks re-shard onto N / 2 (``utils/io.py`` restore_table):
    the restored job dumps exactly the features and weights the saving job held."""
    W = _world(backend)
    saved = _run(backend, _pa_save, W, str(tmp_path))
    half = W // 2
    restored = run_nccl(_pa_restore, half, str(tmp_path)) if backend == "nccl" and half > 1 else \
        run_virtual(_pa_restore, half, str(tmp_path), mode="sync")
    ids_a, w_a = torch.cat([s[0] for s in saved]), torch.cat([s[1] for s in saved])
    ids_b, w_b = torch.cat([s[0] for s in restored]), torch.cat([s[1] for s in restored])
    oa, ob = torch.argsort(ids_a), torch.argsort(ids_b)
    assert ids_a.numel() > 0 and torch.equal(ids_a[oa], ids_b[ob])
    assert torch.equal(w_a[oa], w_b[ob])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("backend", BACKENDS)
@pytest.mark.parametrize("optimizer", ["add", "adagrad"])
def test_capacity_table_bounded_staleness_equals_host_synchronous_world(backend, optimizer):
    """BASELINE config #5 (the sharded embedding table with bounded staleness 2) on N
    ranks vs the host-synchronous world: the same shards to fp32 summation order and
    the same pushed rows; the loss falls."""
    W = _world(backend) if backend == "nccl" else 8
    res = _run(backend, _pair_emb, W, optimizer)
    ref = run_virtual(_pair_emb, W, optimizer, mode="sync")
    # adagrad: a hot key's accumulated squares differ in the last bits between runs (float
    # atomics sum its per-source gradients in any order), and 1 / sqrt(G) amplifies that in
    # its later steps (measured: 2 of 16M elements at 2e-5); a lost or doubled push moves a
    # row by ~lr = 5e-2
    tol = dict(rtol=1e-3, atol=1e-4) if optimizer == "adagrad" else dict(rtol=1e-4, atol=1e-5)
    for (wa, l0a, l1a, ra), (wb, l0b, l1b, rb) in zip(res, ref):
        assert ra == rb and l1a < l0a
        torch.testing.assert_close(wa, wb, **tol)


def _graph_step(comm, graph):
    """Fixed-shape plans at world N (keys / rows / deltas: three all-to-alls per micro-batch);
    ``graph=True`` captures the whole step -- its RCCL all-to-alls included -- into one
    hipGraph and replays it (``core/step_graph.py``)."""
    from flink_parameter_server_1_amd.api.batched import BatchedWorkerLogic
    from flink_parameter_server_1_amd.core.tensor_engine import TensorRuntime
    from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogic

    class W(BatchedWorkerLogic):
        graph_safe = True

        def on_recv_batch(self, batch, ps):
            keys, w = batch
            ps.pull(keys, payload=w)

        def on_pull_recv_batch(self, pulled, ps):
            ps.push(0.1 * pulled.values() + pulled.payload.view(-1, 1))

    logic = DeviceSimplePSLogic(5000, 8, op="add", init=("uniform", -0.1, 0.1), seed=3)
    rt = TensorRuntime(comm, staleness=0, graph=graph, capacity=512).start(W(), logic)
    g = torch.Generator(device=comm.device).manual_seed(11 + comm.rank)
    for _ in range(10):
        rt.submit((torch.randint(0, 5000, (256,), generator=g, device=comm.device),
                   torch.rand(256, generator=g, device=comm.device)))
    rt.finish()
    torch.cuda.synchronize()
    replays = rt.graphs.replays if graph and rt.graphs is not None else 0
    return logic.table.weight.cpu(), replays


@pytest.mark.timeout(600)
@pytest.mark.skipif(N_GPUS < 2, reason="needs >= 2 GPUs")
def test_graph_captured_rccl_step_equals_eager_across_gpus():
    """What the one-rank loopback group could not show: a hipGraph holding RCCL
    all-to-alls between DIFFERENT GPUs replays to the eager engine's tables."""
    eager = run_nccl(_graph_step, N_GPUS, False)
    graph = run_nccl(_graph_step, N_GPUS, True)
    for (w0, _), (w1, replays) in zip(eager, graph):
        assert replays > 0
        torch.testing.assert_close(w1, w0, rtol=1e-5, atol=1e-5)


@pytest.mark.timeout(600)
def test_verify_sees_a_missing_stream_wait():
    """The check itself under RCCL semantics: the rotation with the ``w.wait()`` of
    ``RingRotation.end`` removed (sub-steps on one stream) fails it; the intact one passes."""
    from test_vworld_gpu import _load_mutant

    from flink_parameter_server_1_amd.parallel.verify import rotation_check

    mutant = _load_mutant("                w.wait()\n")

    def body(comm, cls):
        return rotation_check(comm, schedule="bidir", overlap=False, rotation_cls=cls)

    good = run_virtual(body, 4, None, mode="async", latency_us=1000.0)
    bad = run_virtual(body, 4, mutant.RingRotation, mode="async", latency_us=1000.0)
    assert all(r["verify_ok"] for r in good)
    assert not any(r["verify_ok"] for r in bad)
