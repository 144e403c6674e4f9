"""hipGraph-replayed tensor-engine steps (``core.step_graph``): results equal the
eager engine exactly; shape changes, workspace reuse and a syncing worker."""
import warnings

import pytest
import torch

from flink_parameter_server_1_amd.api.batched import BatchedWorkerLogic, FunctionBatchedWorkerLogic
from flink_parameter_server_1_amd.core.tensor_engine import FoldSink, TensorRuntime
from flink_parameter_server_1_amd.parallel.comm import Comm
from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogic, DeviceSimplePSLogicWithClose

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
KEYS, DIM = 5000, 8


class _Worker(BatchedWorkerLogic):
    """Pulls the batch's keys, pushes 0.1 * value + weight per request, emits the
    pulled values of the first 3 requests as a Left output."""

    graph_safe = True

    def on_recv_batch(self, batch, ps):
        keys, w = batch
        ps.pull(keys, payload=w)

    def on_pull_recv_batch(self, pulled, ps):
        v = pulled.values()
        ps.push(0.1 * v + pulled.payload.view(-1, 1))
        ps.output((pulled.keys[:3], v[:3]))


def _batches(sizes, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    out = []
    for n in sizes:
        keys = torch.randint(0, 300, (n,), generator=g, device=DEV)  # many repeats
        out.append((keys, torch.rand(n, generator=g, device=DEV)))
    return out


def _run(batches, graph, logic_cls=DeviceSimplePSLogic, capacity=None, loopback=False):
    sink = FoldSink(KEYS, DIM, device=DEV)
    lefts = []

    def on(e):
        sink(e)
        if type(e).__name__ == "Left":
            lefts.append(tuple(t.clone() for t in e.value))

    logic = logic_cls(KEYS, DIM, op="add", init=("uniform", -0.1, 0.1), seed=3)
    comm = Comm(device=DEV)
    comm.loopback = loopback
    rt = TensorRuntime(comm, staleness=0, output_sink=on, graph=graph, capacity=capacity).start(_Worker(), logic)
    for b in batches:
        rt.submit(b)
    rt.finish()
    torch.cuda.synchronize()
    return logic.table.weight.clone(), sink, lefts, rt


def test_graph_replay_equals_eager():
    batches = _batches([256] * 12)
    w0, s0, l0, _ = _run(batches, graph=False)
    w1, s1, l1, rt = _run(batches, graph=True)
    assert rt.graphs.disabled is None, rt.graphs.disabled_trace
    assert rt.graphs.captures == 1 and rt.graphs.replays == 12 - 2
    # duplicate keys are summed by float atomics (index_add_): equal up to summation order
    torch.testing.assert_close(w1, w0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(s1.tables["right"], s0.tables["right"], rtol=1e-5, atol=1e-5)
    assert torch.equal(s1.seen["right"], s0.seen["right"])
    assert len(l1) == len(l0) == 12
    for a, b in zip(l0, l1):
        assert torch.equal(a[0], b[0])
        torch.testing.assert_close(a[1], b[1], rtol=1e-5, atol=1e-5)
    assert rt.counters.c["micro_batches"] == 12
    assert rt.ps_logic.ps.stats["steps"] == 12


def test_graph_shapes_and_close_dump():
    """Two interleaved batch shapes -> two graphs; the close-time dump (touched rows)
    matches the eager run."""
    batches = _batches([64, 128] * 6, seed=1)
    w0, s0, _, _ = _run(batches, graph=False, logic_cls=DeviceSimplePSLogicWithClose)
    w1, s1, _, rt = _run(batches, graph=True, logic_cls=DeviceSimplePSLogicWithClose)
    assert rt.graphs.captures == 2
    torch.testing.assert_close(w1, w0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(s1.tables["right"], s0.tables["right"], rtol=1e-5, atol=1e-5)
    assert torch.equal(s1.seen["right"], s0.seen["right"])


def test_graph_needs_graph_safe_worker():
    w = FunctionBatchedWorkerLogic(lambda b, ps: ps.pull(b), lambda p, ps: None)
    with pytest.raises(ValueError, match="graph_safe"):
        TensorRuntime(Comm(device=DEV), graph=True).start(w, DeviceSimplePSLogic(KEYS, DIM))


def test_syncing_worker_falls_back_to_eager():
    """A worker that syncs inside its callback: the capture fails, the runtime warns
    and runs eagerly, and the results still equal the eager run."""

    def answer(pulled, ps):
        if float(pulled.values().sum().item()) > 1e30:  # host sync
            raise AssertionError
        ps.push(torch.ones_like(pulled.values()))

    batches = [b[0] for b in _batches([128] * 6, seed=2)]
    tables = []
    for graph in (False, True):
        logic = DeviceSimplePSLogicWithClose(KEYS, DIM, op="add")
        w = FunctionBatchedWorkerLogic(lambda b, ps: ps.pull(b), answer, graph_safe=True)
        rt = TensorRuntime(Comm(device=DEV), output_sink=lambda e: None, graph=graph).start(w, logic)
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            for b in batches:
                rt.submit(b)
        rt.finish()
        if graph:
            assert rt.graphs.disabled is not None and rt.graphs.replays == 0
            assert any("capture disabled" in str(r.message) for r in rec)
        tables.append(logic.table.weight.clone())
    torch.testing.assert_close(tables[1], tables[0], rtol=1e-5, atol=1e-5)


def test_graph_replay_captures_rccl_collectives(rccl_loopback):
    """The world > 1 step shape: fixed-shape plans whose key / row / delta all-to-alls
    go through RCCL, captured into the hipGraph with the kernels around them.  Eager
    and replayed steps equal the world-1 static plans' results."""
    batches = _batches([256] * 12, seed=4)
    w0, s0, l0, _ = _run(batches, graph=False)
    w1, s1, l1, rt1 = _run(batches, graph=False, capacity=256, loopback=True)
    w2, s2, l2, rt2 = _run(batches, graph=True, capacity=256, loopback=True)
    assert rt1.ps_logic.ps.fixed() and rt2.ps_logic.ps.fixed()
    assert rt2.graphs.disabled is None, rt2.graphs.disabled_trace
    assert rt2.graphs.captures == 1 and rt2.graphs.replays == 12 - 2
    for w, s, lefts in ((w1, s1, l1), (w2, s2, l2)):
        torch.testing.assert_close(w, w0, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(s.tables["right"], s0.tables["right"], rtol=1e-5, atol=1e-5)
        assert torch.equal(s.seen["right"], s0.seen["right"])
        assert len(lefts) == 12
        for a, b in zip(l0, lefts):
            assert torch.equal(a[0], b[0])
            torch.testing.assert_close(a[1], b[1], rtol=1e-5, atol=1e-5)


def test_graph_execute_ends_on_lagged_flags(rccl_loopback):
    """``execute()`` with captured RCCL steps: the end-of-input flags are read from the
    replayed steps' buffers one micro-batch late, and the job still ends with the
    eager model."""
    batches = _batches([128] * 8, seed=5)
    models = []
    for graph in (False, True):
        logic = DeviceSimplePSLogicWithClose(KEYS, DIM, op="add", init=("uniform", -0.1, 0.1), seed=3)
        comm = Comm(device=DEV)
        comm.loopback = True
        rt = TensorRuntime(comm, output_sink=lambda e: None, graph=graph, capacity=128)
        rt.execute(batches, _Worker(), logic)
        if graph:
            assert rt.graphs.replays >= 5 and rt.graphs.disabled is None
        models.append(logic.table.weight.clone())
    torch.testing.assert_close(models[1], models[0], rtol=1e-5, atol=1e-5)
