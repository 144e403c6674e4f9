"""Port of T/SenderReceiverTest.scala (timer intervals scaled 5 s -> 0.3 s)."""
import time

from flink_parameter_server_1_amd.core.adapters import (CombinationWorkerSender, CountClientSender,
                                                        SimpleWorkerSender, TimerClientSender, all_of, any_of,
                                                        wait_until)

T = 0.3


class Sink:
    def __init__(self):
        self.pulls = {}
        self.pushes = {}

    def simple(self, m):
        self._one(m)

    def array(self, arr):
        for m in arr:
            self._one(m)

    def _one(self, m):
        if m.msg.is_left:
            self.pulls[m.worker_partition_index] = m.msg.value
        else:
            self.pushes[m.worker_partition_index] = m.msg.value


def test_simple_sender():
    s, snd = Sink(), SimpleWorkerSender()
    for i in range(1, 4):
        snd.on_pull(i, s.simple, i)
    for i in range(4, 11):
        snd.on_push(i, float(i), s.simple, i)
    assert sorted(s.pulls) == [1, 2, 3] and sorted(s.pushes) == list(range(4, 11))


def test_counter_sender():
    s = Sink()
    snd = CombinationWorkerSender(lambda cs: cs[0].should_send(), [CountClientSender(3)])
    for i in (1, 2):
        snd.on_pull(i, s.array, i)
    assert not s.pulls and not s.pushes
    snd.on_pull(3, s.array, 3)
    assert len(s.pulls) == 3
    for i in (1, 2, 3):
        snd.on_push(i, float(i), s.array, i)
    assert len(s.pushes) == 3
    snd.on_push(4, 4.0, s.array, 4)
    assert len(s.pushes) == 3


def test_timer_sender():
    s = Sink()
    snd = CombinationWorkerSender(lambda cs: cs[0].should_send(), [TimerClientSender(T)])
    snd.on_pull(1, s.array, 1)
    assert len(s.pulls) == 0
    assert wait_until(lambda: len(s.pulls) == 1, 4 * T)
    s.pulls.clear()
    for i in range(1, 6):
        snd.on_pull(i, s.array, i)
        snd.on_push(i, float(i), s.array, i)
    assert wait_until(lambda: len(s.pulls) == 5 and len(s.pushes) == 5, 4 * T)
    snd.close()


def test_count_or_timer():
    s = Sink()
    snd = CombinationWorkerSender(any_of, [CountClientSender(5), TimerClientSender(T)])
    for i in range(1, 5):
        snd.on_push(i, float(i), s.array, i)
    assert len(s.pushes) == 0
    snd.on_push(5, 5.0, s.array, 5)
    assert len(s.pushes) == 5
    snd.on_pull(1, s.array, 1)
    assert len(s.pulls) == 0
    assert wait_until(lambda: len(s.pulls) == 1, 4 * T)
    snd.close()


def test_count_and_timer():
    s = Sink()
    snd = CombinationWorkerSender(all_of, [CountClientSender(5), TimerClientSender(T)])
    snd.on_pull(1, s.array, 1)
    time.sleep(T + 0.2)
    assert len(s.pulls) == 0
    for i in range(1, 6):
        snd.on_push(i, float(i), s.array, i)
    # the buffer held pull + 5 pushes; the count fired on the 4th push (pull counted)
    assert wait_until(lambda: len(s.pulls) == 1 and len(s.pushes) == 4, 2 * T)
    snd.close()
