"""Ports of T/utils/FlinkEOFTest.scala and T/utils/FlinkSleepBlockerTest.scala.

EOF: 7 source subtasks x 5 records, each source emitting its own index and
sleeping ``index * d`` before every record (so sources finish at different
times); the downstream subtask must see every record before ``on_eof`` and
report ``sum = 5 * (0 + ... + 6) = 105`` (``FlinkEOFTest.scala:17,65,77``).
Sleep blocker: the blocked record arrives 0.9-1.5 x the block delay after the
non-blocked one (``FlinkSleepBlockerTest.scala:10,51-52``); the delay is 0.5 s
here instead of 5 s to keep the suite fast.
"""
import threading
import time

import pytest

from flink_parameter_server_1_amd.core.engine import PartitionedInput
from flink_parameter_server_1_amd.core.messages import Left, Right
from flink_parameter_server_1_amd.models.mf.apps import OnlineFactorModelBuilder
from flink_parameter_server_1_amd.models.mf.core import IDGenerator
from flink_parameter_server_1_amd.utils.eof import (EOF, IllegalStateException, flat_map_with_eof, flatMapWithEOF,
                                                     with_eof)
from flink_parameter_server_1_amd.utils.sleep_blocker import block, block_partitions

RECORDS_PER_SOURCE = 5
SRC_PARALLELISM = 7


def _source(idx, sleep_s):
    for _ in range(RECORDS_PER_SOURCE):
        time.sleep(idx * sleep_s)
        yield idx


class _SumUntilEOF:
    def __init__(self):
        self.is_eof = False
        self.sum = 0
        self.ctx = None

    def open(self, ctx):
        self.ctx = ctx

    def flat_map(self, value, collect):
        assert not self.is_eof, "Should not have received input after EOF"
        n = self.ctx.number_of_parallel_subtasks
        assert value % n == self.ctx.index_of_this_subtask, "Unexpected record at subtask"
        self.sum += value

    def on_eof(self, collect):
        self.is_eof = True
        collect(f"EOF {self.sum}")


@pytest.mark.parametrize("parallelism", [1, 3])
def test_eof_barrier_sum(parallelism):
    sources = [_source(i, 0.01) for i in range(SRC_PARALLELISM)]
    outs = flat_map_with_eof(sources, _SumUntilEOF(), parallelism, partitioner=lambda k, n: k % n)
    assert all(len(o) == 1 and o[0].startswith("EOF ") for o in outs)
    total = sum(int(o[0].split()[1]) for o in outs)
    assert total == sum(range(SRC_PARALLELISM)) * RECORDS_PER_SOURCE == 105


def test_eof_per_subtask_sums():
    sources = [_source(i, 0.0) for i in range(SRC_PARALLELISM)]
    outs = flatMapWithEOF(sources, _SumUntilEOF(), 3, partitioner=lambda k, n: k % n)
    for t, o in enumerate(outs):
        assert o == [f"EOF {RECORDS_PER_SOURCE * sum(i for i in range(SRC_PARALLELISM) if i % 3 == t)}"]


def test_eof_empty_source_raises():
    with pytest.raises(IllegalStateException):
        flat_map_with_eof([[1, 2], []], _SumUntilEOF(), 1, partitioner=lambda k, n: 0)


def test_with_eof_appends_marker_to_every_partition():
    inp = with_eof(list(range(10)), 3)
    assert isinstance(inp, PartitionedInput) and len(inp.parts) == 3
    seen = []
    for p in inp.parts:
        assert p[-1] == Left(EOF())
        assert all(isinstance(x, Right) for x in p[:-1])
        seen += [x.value for x in p[:-1]]
    assert sorted(seen) == list(range(10))


def test_sleep_blocker_delays_first_record():
    block_ms = 500
    arrivals = {}
    lock = threading.Lock()

    def drain(stream, name):
        for _ in stream:
            with lock:
                arrivals.setdefault(name, time.monotonic())

    started = {}

    def drain_timed(stream, name):
        started.setdefault(name, time.monotonic())  # the stream's own first iteration
        drain(stream, name)

    blocked = [block(["blocked"], block_ms) for _ in range(2)]
    non_blocked = [["nonBlocked"] for _ in range(3)]
    threads = [threading.Thread(target=drain_timed, args=(s, "blocked")) for s in blocked]
    threads += [threading.Thread(target=drain_timed, args=(s, "nonBlocked")) for s in non_blocked]
    for th in threads:
        th.start()
    for th in threads:
        th.join(10)
    assert arrivals["nonBlocked"] < arrivals["blocked"]
    # the blocked stream's delay measured from its own start (thread scheduling
    # jitter between threads does not enter); generous upper bound for loaded hosts
    delay_ms = (arrivals["blocked"] - started["blocked"]) * 1000
    assert block_ms * 0.9 < delay_ms < block_ms * 3.0


def test_sleep_blocker_is_lazy_and_blocks_once():
    t0 = time.monotonic()
    s = block(range(5), 200)
    assert time.monotonic() - t0 < 0.1  # nothing happens until iteration starts
    it = iter(s)
    assert next(it) == 0
    assert time.monotonic() - t0 >= 0.18
    t1 = time.monotonic()
    assert list(it) == [1, 2, 3, 4]
    assert time.monotonic() - t1 < 0.1


def test_block_partitions():
    inp = block_partitions(PartitionedInput([[1, 2], [3]]), 50)
    t0 = time.monotonic()
    assert [list(p) for p in inp.parts] == [[1, 2], [3]]
    assert time.monotonic() - t0 >= 0.09


def test_id_generator_monotonic_and_builder_is_abstract():
    a, b = IDGenerator.next(), IDGenerator.next()
    assert b == a + 1
    with pytest.raises(NotImplementedError):
        OnlineFactorModelBuilder().buildModel([], None, None, {})
