"""Ports of T/server/SimplePSLogicTest.scala, LockPSLogicATest.scala, LockPSLogicBTest.scala."""
import pytest

from flink_parameter_server_1_amd import (LockPSLogicA, LockPSLogicB, ParameterServer, RangePSLogicWithClose,
                                          RuntimeContext, SimplePSLogic, SimplePSLogicWithClose)
from flink_parameter_server_1_amd.ps import IllegalStateException, range_shard_bounds


class MockPS(ParameterServer):
    def __init__(self):
        self.answers = []
        self.outputs = []

    def answer_pull(self, pid, value, widx):
        self.answers.append((pid, value, widx))

    def output(self, out):
        self.outputs.append(out)


def test_simple_ps_lazy_init_and_push_output():
    logic = SimplePSLogic(lambda x: 23, lambda x, y: x + y)
    ps = MockPS()
    logic.on_pull_recv(42, 1, ps)
    assert logic.params[42] == 23
    assert ps.answers == [(42, 23, 1)]
    logic.on_push_recv(42, 0, ps)
    assert ps.outputs == [(42, 23)]


def test_simple_ps_push_before_pull_sets_delta():
    logic = SimplePSLogic(lambda x: 100, lambda x, y: x + y)
    ps = MockPS()
    logic.on_push_recv(7, 5, ps)
    assert logic.params[7] == 5 and ps.outputs == [(7, 5)]


def test_simple_ps_with_close_dumps_at_close():
    logic = SimplePSLogicWithClose(lambda x: 0, lambda x, y: x + y)
    ps = MockPS()
    logic.on_pull_recv(1, 0, ps)
    logic.on_push_recv(1, 3, ps)
    logic.on_push_recv(2, 4, ps)
    assert ps.outputs == []
    logic.close(ps)
    assert sorted(ps.outputs) == [(1, 3), (2, 4)]


def test_range_ps_bounds_and_dump():
    assert range_shard_bounds(10, 3, 0) == (0, 4)
    assert range_shard_bounds(10, 3, 2) == (8, 2)
    logic = RangePSLogicWithClose(10, lambda i: float(i), lambda a, b: a + b)
    logic.open({}, RuntimeContext(1, 3))
    ps = MockPS()
    logic.on_pull_recv(5, 0, ps)
    assert ps.answers == [(5, 5.0, 0)]
    logic.on_push_recv(5, 1.0, ps)
    logic.on_push_recv(6, 2.0, ps)
    logic.close(ps)
    assert ps.outputs == [(5, 6.0), (6, 2.0)]
    with pytest.raises(IndexError):
        logic.on_pull_recv(0, 0, ps)


@pytest.mark.parametrize("cls", [LockPSLogicA, LockPSLogicB])
def test_lock_push_without_pull_throws(cls):
    logic = cls(lambda x: x, lambda x, y: x)
    with pytest.raises(IllegalStateException):
        logic.on_push_recv(42, 42, MockPS())


@pytest.mark.parametrize("cls", [LockPSLogicA, LockPSLogicB])
def test_lock_init(cls):
    logic = cls(lambda x: 23, lambda x, y: y)
    logic.on_pull_recv(42, 42, MockPS())
    assert logic.params[42][1] == 23


@pytest.mark.parametrize("cls", [LockPSLogicA, LockPSLogicB])
def test_lock_update_after_push(cls):
    logic = cls(lambda x: 0, lambda x, y: y)
    logic.on_pull_recv(42, 42, MockPS())
    ps = MockPS()
    logic.on_push_recv(42, 23, ps)
    assert ps.outputs[-1] == (42, 23)


@pytest.mark.parametrize("cls", [LockPSLogicA, LockPSLogicB])
def test_locking_queues_second_puller(cls):
    logic = cls(lambda x: 0, lambda x, y: y)
    logic.on_pull_recv(42, 42, MockPS())
    ps = MockPS()
    logic.on_pull_recv(42, 43, ps)
    assert ps.answers == []
    locked, param, q = logic.params[42]
    assert locked and param == 0 and list(q) == [43]


@pytest.mark.parametrize("cls", [LockPSLogicA, LockPSLogicB])
def test_lock_released(cls):
    logic = cls(lambda x: 0, lambda x, y: y)
    logic.on_pull_recv(42, 42, MockPS())
    logic.on_push_recv(42, 23, MockPS())
    locked, param, q = logic.params[42]
    assert not locked and param == 23 and len(q) == 0


@pytest.mark.parametrize("cls", [LockPSLogicA, LockPSLogicB])
def test_lock_held_answers_next(cls):
    logic = cls(lambda x: 0, lambda x, y: y)
    logic.on_pull_recv(42, 42, MockPS())
    logic.on_pull_recv(42, 43, MockPS())
    ps = MockPS()
    logic.on_push_recv(42, 23, ps)
    assert ps.answers == [(42, 23, 43)]
    locked, param, q = logic.params[42]
    assert locked and param == 23 and len(q) == 0


def test_lock_a_duplicates_queue_twice():
    logic = LockPSLogicA(lambda x: 0, lambda x, y: y)
    for w in (42, 43, 43):
        logic.on_pull_recv(42, w, MockPS())
    locked, param, q = logic.params[42]
    assert locked and param == 0 and list(q) == [43, 43]


def test_lock_b_deduplicates_queue():
    logic = LockPSLogicB(lambda x: 0, lambda x, y: y)
    for w in (42, 43, 43):
        logic.on_pull_recv(42, w, MockPS())
    locked, param, q = logic.params[42]
    assert locked and list(q) == [43]


def test_lock_b_dedup_with_push():
    logic = LockPSLogicB(lambda x: 0, lambda x, y: x + y)
    for w in (42, 43, 43, 44):
        logic.on_pull_recv(42, w, MockPS())
    ps = MockPS()
    logic.on_push_recv(42, 5, ps)
    assert ps.answers == [(42, 5, 43)]
    logic.on_pull_recv(42, 43, MockPS())
    _, param, q = logic.params[42]
    assert list(q) == [44, 43] and param == 5
