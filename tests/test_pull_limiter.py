"""Port of T/WorkerLogicTest.scala (+ blocking limiter and future client, untested upstream)."""
import threading
import time

from flink_parameter_server_1_amd import (ParameterServerClient, WorkerLogic, WorkerLogicWithFuture,
                                          add_blocking_pull_limiter, add_pull_limiter)


class _Worker(WorkerLogic):
    def on_recv(self, data, ps):
        ps.pull(data)

    def on_pull_recv(self, param_id, value, ps):
        pass


class _CountingPS(ParameterServerClient):
    def __init__(self):
        self.pull_counter = 0
        self.pushes = []

    def pull(self, param_id):
        self.pull_counter += 1

    def push(self, param_id, delta):
        self.pushes.append((param_id, delta))

    def output(self, out):
        pass


def test_pull_limiter_limits_pulls():
    ps = _CountingPS()
    limited = add_pull_limiter(_Worker(), 10)
    for x in range(1, 21):
        limited.on_recv(x, ps)
    assert ps.pull_counter == 10
    for x in range(1, 6):
        limited.on_pull_recv(x, -1, ps)
    assert ps.pull_counter == 15
    limited.on_recv(21, ps)
    assert ps.pull_counter == 15
    for x in range(6, 22):
        limited.on_pull_recv(x, -1, ps)
    assert ps.pull_counter == 21


def test_scala_spelling_worker():
    class ScalaWorker(WorkerLogic):
        def onRecv(self, data, ps):  # noqa: N802
            ps.pull(data)

        def onPullRecv(self, pid, v, ps):  # noqa: N802
            ps.push(pid, v)

    ps = _CountingPS()
    w = add_pull_limiter(ScalaWorker(), 2)
    w.on_recv(1, ps)
    w.on_pull_recv(1, 5, ps)
    assert ps.pull_counter == 1 and ps.pushes == [(1, 5)]


def test_blocking_pull_limiter_blocks_foreign_thread():
    ps = _CountingPS()
    limited = add_blocking_pull_limiter(_Worker(), 3)
    limited._set_ps(ps)
    done = threading.Event()

    def puller():
        for x in range(5):
            limited._client.pull(x)
        done.set()

    t = threading.Thread(target=puller, daemon=True)
    t.start()
    time.sleep(0.2)
    assert ps.pull_counter == 3 and not done.is_set()
    limited.on_pull_recv(0, 0, ps)
    limited.on_pull_recv(1, 0, ps)
    assert done.wait(2.0)
    assert ps.pull_counter == 5


def test_future_worker_completes_in_fifo_order():
    seen = []

    class FW(WorkerLogicWithFuture):
        def on_data_recv(self, data, ps):
            f = ps.pull(data % 2)
            f.on_complete(lambda ans: seen.append((data, ans)))

    ps = _CountingPS()
    w = FW()
    for d in [0, 1, 2]:
        w.on_recv(d, ps)
    assert ps.pull_counter == 3
    w.on_pull_recv(0, "a", ps)
    w.on_pull_recv(1, "b", ps)
    w.on_pull_recv(0, "c", ps)
    assert seen == [(0, (0, "a")), (1, (1, "b")), (2, (0, "c"))]
