"""Integration tests of the engine — ports of T/FlinkSimpleStackTest.scala,
T/FlinkParameterServerTest.scala and T/FlinkCombinationStackTest.scala, with
assertions added where the reference only printed."""
import numpy as np
import pytest

from flink_parameter_server_1_amd import (LogicFactory, ParameterServerLogic, SimplePSLogic, SimplePSLogicWithClose,
                                          WorkerLogic, transform, transform_with_double_model_load,
                                          transform_with_model_load)
from flink_parameter_server_1_amd.api import BaseMFWorkerLogic
from flink_parameter_server_1_amd.core.adapters import (CombinationPSSender, CombinationWorkerSender,
                                                        CountClientSender, CountPSSender, MultiplePSReceiver,
                                                        MultipleWorkerReceiver, PSReceiver, PSSender,
                                                        TimerClientSender, TimerPSSender, WorkerReceiver,
                                                        WorkerSender, all_of, any_of)
from flink_parameter_server_1_amd.core.messages import PullAnswer, left_values, right_values


class AddWorker(WorkerLogic):
    """Pull a row id, push the record's vector as delta (FlinkSimpleStackTest shape)."""

    def __init__(self):
        self.waiting = {}

    def on_recv(self, data, ps):
        rid, vec = data
        self.waiting.setdefault(rid, []).append(vec)
        ps.pull(rid)

    def on_pull_recv(self, pid, value, ps):
        delta = self.waiting[pid].pop(0)
        ps.push(pid, delta)
        ps.output((pid, tuple(value)))


DATA = [(1, (1.5, 5.3, 1.3, 5.6, 7.9)), (2, (0.1,) * 5), (2, (10.1, 10.2, 10.3, 10.4, 10.5)),
        (3, (20.5, 26.3, 28.1, 29.2, 29.7)), (5, (100.0, 101, 102, 103, 104)), (4, (4.5, 9.6, 2.3, 9.9, 0.5)),
        (5, (4.8, 15, 16, 23, 42)), (1, (1000.0,) * 5)]


def _vsum(a, b):
    return tuple(x + y for x, y in zip(a, b))


@pytest.mark.parametrize("W,P", [(1, 1), (4, 4), (3, 2)])
def test_simple_stack_sums_vectors(W, P):
    out = transform(DATA, AddWorker(), SimplePSLogicWithClose(lambda i: (0.0,) * 5, _vsum),
                    worker_parallelism=W, ps_parallelism=P, data_partitioner=lambda d: d[0])
    final = dict(right_values(out))
    expect = {}
    for rid, vec in DATA:
        expect[rid] = _vsum(expect.get(rid, (0.0,) * 5), vec)
    assert set(final) == set(expect)
    for k in expect:
        np.testing.assert_allclose(final[k], expect[k])
    assert len(left_values(out)) == len(DATA)


def test_overload_a_param_init_update():
    out = transform(DATA, AddWorker(), param_init=lambda i: (0.0,) * 5, param_update=_vsum,
                    worker_parallelism=2, ps_parallelism=2)
    # SimplePSLogic emits on every push
    assert len(right_values(out)) == len(DATA)


class CountingWorker(WorkerLogic):
    """Pull id three times, push +1 each answer (model-load test shape)."""

    def on_recv(self, data, ps):
        ps.pull(data)

    def on_pull_recv(self, pid, value, ps):
        ps.push(pid, 1)


@pytest.mark.parametrize("W,P", [(4, 3), (1, 1), (2, 5)])
def test_model_load_exact(W, P):
    """T/FlinkSimpleStackTest.scala:121-206 — final dump == 10*i + 3."""
    n = 50
    model = [(i, 10 * i) for i in range(n)]
    data = [i for i in range(n) for _ in range(3)]
    out = transform_with_model_load(model, data, CountingWorker(),
                                    SimplePSLogicWithClose(lambda i: 0, lambda a, b: a + b),
                                    worker_parallelism=W, ps_parallelism=P)
    final = dict(right_values(out))
    assert final == {i: 10 * i + 3 for i in range(n)}


def test_model_load_needs_a_param_per_partition():
    with pytest.raises(RuntimeError):
        transform_with_model_load([(0, 1)], [0], CountingWorker(),
                                  SimplePSLogicWithClose(lambda i: 0, lambda a, b: a + b),
                                  worker_parallelism=2, ps_parallelism=1)


class ItemWorker(BaseMFWorkerLogic):
    def on_recv(self, data, ps):
        ps.pull(data)

    def on_pull_recv(self, pid, value, ps):
        ps.output((pid, value, sum(self.model.values())))


def test_double_model_load_routes_left_to_ps_and_right_to_worker():
    from flink_parameter_server_1_amd import Left, Right

    model = [Left((i, 100 + i)) for i in range(6)] + [Right((i, 1)) for i in range(4)]
    out = transform_with_double_model_load(model, [0, 1, 2, 3, 4, 5], ItemWorker(),
                                           SimplePSLogicWithClose(lambda i: -1, lambda a, b: b),
                                           worker_parallelism=2, ps_parallelism=2)
    wouts = left_values(out)
    assert sorted((p, v) for p, v, _ in wouts) == [(i, 100 + i) for i in range(6)]
    # each worker got half of the 4 worker-model records
    assert sorted(s for _, _, s in wouts) == [2] * 6
    assert dict(right_values(out)) == {i: 100 + i for i in range(6)}


def test_custom_wire_format_queue_params():
    """T/FlinkParameterServerTest.scala 'flink mock PS' — tuples/string arrays on the wire."""

    class W_(WorkerLogic):
        def __init__(self):
            self.q = []

        def on_recv(self, data, ps):
            self.q.append(data)
            ps.pull(data % 2)

        def on_pull_recv(self, pid, value, ps):
            xs = [x for x in self.q if x % 2 == pid]
            self.q = [x for x in self.q if x % 2 != pid]
            ps.push(pid, xs)

    class PSL(ParameterServerLogic):
        def __init__(self):
            self.params = {}

        def on_pull_recv(self, pid, widx, ps):
            ps.answer_pull(pid, self.params.setdefault(pid, []), widx)

        def on_push_recv(self, pid, delta, ps):
            self.params[pid].extend(delta)
            ps.output(",".join(map(str, self.params[pid])))

    class WR(WorkerReceiver):
        def on_pull_answer_recv(self, msg, handler):
            handler(PullAnswer(msg[0], [int(x) for x in msg[1][1:]]))

    class WS(WorkerSender):
        def on_pull(self, pid, collect, part):
            collect((True, (part, pid)))

        def on_push(self, pid, delta, collect, part):
            collect((False, (pid, *delta)))

    class PR(PSReceiver):
        def on_worker_msg(self, msg, on_pull, on_push):
            if msg[0]:
                on_pull(msg[1][1], msg[1][0])
            else:
                on_push(msg[1][0], list(msg[1][1:]))

    class PSS(PSSender):
        def on_pull_answer(self, pid, value, widx, collect):
            collect((pid, [str(widx)] + [str(v) for v in value]))

    data = [0, 1, 2, 3, 4, 5, 6, 7, 9]
    out = transform(data, W_(), PSL(),
                    param_partitioner=lambda m: abs(m[1][1] if m[0] else m[1][0]),
                    w_in_partition=lambda m: int(m[1][0]),
                    worker_parallelism=4, ps_parallelism=4,
                    worker_receiver=WR(), worker_sender=WS(), ps_receiver=PR(), ps_sender=PSS())
    ps_out = right_values(out)
    evens = max((s for s in ps_out if s and int(s.split(",")[0]) % 2 == 0), key=len)
    odds = max((s for s in ps_out if s and int(s.split(",")[0]) % 2 == 1), key=len)
    assert sorted(map(int, evens.split(","))) == [0, 2, 4, 6]
    assert sorted(map(int, odds.split(","))) == [1, 3, 5, 7, 9]


def test_combination_stack_count_and_timer():
    """T/FlinkCombinationStackTest.scala — client Count(4) AND Timer, PS Count OR Timer."""
    csend = CombinationWorkerSender(all_of, [CountClientSender(4), TimerClientSender(0.05)])
    psend = CombinationPSSender(any_of, [CountPSSender(4), TimerPSSender(0.05)])
    out = transform(DATA, AddWorker(), SimplePSLogic(lambda i: (0.0,) * 5, _vsum),
                    param_partitioner=lambda arr: arr[0].worker_partition_index,
                    w_in_partition=lambda arr: arr[0].worker_partition_index % 4 if arr else 0,
                    worker_parallelism=4, ps_parallelism=4,
                    worker_receiver=MultipleWorkerReceiver(), worker_sender=csend,
                    ps_receiver=MultiplePSReceiver(), ps_sender=psend,
                    data_partitioner=lambda d: d[0], iteration_wait_time=300)
    assert len(left_values(out)) == len(DATA)
    # rows are keyed by data partition; every vector was pushed once
    total = np.zeros(5)
    last = {}
    for pid, v in right_values(out):
        last[pid] = v
    for v in last.values():
        total += np.array(v)
    np.testing.assert_allclose(total, np.sum([v for _, v in DATA], axis=0))


def test_logic_factory_builds_per_subtask():
    made = []

    def make(i):
        made.append(i)
        return AddWorker()

    transform(DATA, LogicFactory(make), SimplePSLogicWithClose(lambda i: (0.0,) * 5, _vsum), worker_parallelism=3)
    assert sorted(made) == [0, 1, 2]
