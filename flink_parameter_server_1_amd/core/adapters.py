"""L2 transport adapters: wire encoding and message combining.

Traits (``M/FlinkParameterServer.scala:942-987``):

* ``WorkerSender.on_pull(id, collect, partition_id)`` /
  ``on_push(id, delta, collect, partition_id)``
* ``WorkerReceiver.on_pull_answer_recv(msg, pull_handler)``
* ``PSSender.on_pull_answer(id, value, worker_idx, collect)``
* ``PSReceiver.on_worker_msg(msg, on_pull_recv, on_push_recv)``

Implementations:

* Simple* — one message per record (``M/client/sender/SimpleWorkerSender.scala``,
  ``M/client/receiver/SimpleWorkerReceiver.scala``, ``M/server/sender/SimplePSSender.scala``,
  ``M/server/receiver/SimplePSReceiver.scala``).
* Multiple* — decode list batches (``M/client/receiver/MultipleWorkerReceiver.scala``,
  ``M/server/receiver/MultiplePSReceiver.scala``).
* Combination* — micro-batching senders driven by ``Combinable`` flags
  (``M/common/{Combinable,CombinationLogic,CountLogic,TimerLogic}.scala``,
  ``M/client/sender/CombinationWorkerSender.scala``,
  ``M/server/sender/CombinationPSSender.scala``).  A user predicate over the
  flags (AND / OR ...) decides when the whole buffer is flushed as one list.

Design difference: the reference's timer thread appends/flushes
the same buffer as the operator thread without synchronisation.  Here the
buffer is guarded by a re-entrant lock and the engine's collectors are
thread-safe, so a timer flush can never race an append.  Timer threads are
daemons and are stopped by ``close()``.
"""
from __future__ import annotations

import threading
import time
from typing import Callable, List

from .messages import Left, Pull, PullAnswer, Push, PSToWorker, Right, WorkerToPS


# ---------------------------------------------------------------- traits
class WorkerSender:
    def on_pull(self, param_id, collect, partition_id):
        raise NotImplementedError

    def on_push(self, param_id, delta, collect, partition_id):
        raise NotImplementedError

    def close(self):
        pass

    def pending(self) -> int:
        return 0



class WorkerReceiver:
    def on_pull_answer_recv(self, msg, pull_handler):
        raise NotImplementedError


class PSSender:
    def on_pull_answer(self, param_id, value, worker_partition_index, collect):
        raise NotImplementedError

    def close(self):
        pass

    def pending(self) -> int:
        return 0


class PSReceiver:
    def on_worker_msg(self, msg, on_pull_recv, on_push_recv):
        raise NotImplementedError


# ---------------------------------------------------------------- simple
class SimpleWorkerSender(WorkerSender):
    def on_pull(self, param_id, collect, partition_id):
        collect(WorkerToPS(partition_id, Left(Pull(param_id))))

    def on_push(self, param_id, delta, collect, partition_id):
        collect(WorkerToPS(partition_id, Right(Push(param_id, delta))))


class SimpleWorkerReceiver(WorkerReceiver):
    def on_pull_answer_recv(self, msg, pull_handler):
        pull_handler(msg.msg)


class SimplePSSender(PSSender):
    def on_pull_answer(self, param_id, value, worker_partition_index, collect):
        collect(PSToWorker(worker_partition_index, PullAnswer(param_id, value)))


def _dispatch_worker_msg(w2ps, on_pull_recv, on_push_recv):
    m = w2ps.msg
    inner = m.value
    if m.is_left and isinstance(inner, Pull):
        on_pull_recv(inner.param_id, w2ps.worker_partition_index)
    elif m.is_right and isinstance(inner, Push):
        on_push_recv(inner.param_id, inner.delta)
    else:
        raise RuntimeError("Parameter server received unknown message.")


class SimplePSReceiver(PSReceiver):
    def on_worker_msg(self, msg, on_pull_recv, on_push_recv):
        _dispatch_worker_msg(msg, on_pull_recv, on_push_recv)


# ---------------------------------------------------------------- multiple
class MultipleWorkerReceiver(WorkerReceiver):
    def on_pull_answer_recv(self, msg, pull_handler):
        for ps2w in msg:
            pull_handler(ps2w.msg)


class MultiplePSReceiver(PSReceiver):
    def on_worker_msg(self, msg, on_pull_recv, on_push_recv):
        for w2ps in msg:
            _dispatch_worker_msg(w2ps, on_pull_recv, on_push_recv)


# ---------------------------------------------------------------- combinables
class Combinable:
    """A flag-raising flush condition (``M/common/Combinable.scala:5-27``)."""

    def __init__(self):
        self._send = False

    def send_condition(self) -> bool:
        raise NotImplementedError

    def logic(self, adder, callback, collect):
        raise NotImplementedError

    def should_send(self) -> bool:
        return self._send

    shouldSend = should_send

    def send(self, callback, collect):
        self._send = True
        callback(collect)

    def reset(self):
        self._send = False

    def close(self):
        pass


class CountLogic(Combinable):
    """Raise the flag after ``max`` messages (``M/common/CountLogic.scala:5-29``)."""

    def __init__(self, max_count: int):
        super().__init__()
        self.max = max_count
        self.count = 0

    def send_condition(self):
        return self.count >= self.max

    def logic(self, adder, callback, collect):
        self.count += 1
        if self.send_condition():
            self.send(callback, collect)
            self.count = 0


class TimerLogic(Combinable):
    """Raise the flag every ``interval`` seconds if data arrived
    (``M/common/TimerLogic.scala:6-51``).  ``interval`` is seconds (float)."""

    def __init__(self, interval: float):
        super().__init__()
        self.interval = float(interval)
        self.contains_data = False
        self._thread = None
        self._stop = threading.Event()

    def send_condition(self):
        return self.contains_data

    def _run(self, callback, collect):
        while not self._stop.wait(self.interval):
            if self.send_condition():
                self.send(callback, collect)
                self.contains_data = False

    def logic(self, adder, callback, collect):
        self.contains_data = True
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, args=(callback, collect), daemon=True)
            self._thread.start()

    def close(self):
        self._stop.set()

    def __deepcopy__(self, memo):
        return type(self)(self.interval)


# client / server flavoured names of the reference
class CountClientSender(CountLogic):
    pass


class CountPSSender(CountLogic):
    pass


class TimerClientSender(TimerLogic):
    pass


class TimerPSSender(TimerLogic):
    pass


def all_of(combinables: List[Combinable]) -> bool:
    return all(c.should_send() for c in combinables)


def any_of(combinables: List[Combinable]) -> bool:
    return any(c.should_send() for c in combinables)


class CombinationLogic:
    """Buffer + flush engine (``M/common/CombinationLogic.scala:6-35``)."""

    def __init__(self, condition: Callable[[List[Combinable]], bool], combinables: List[Combinable]):
        self.condition = condition
        self.combinables = list(combinables)
        self.data: list = []
        self._lock = threading.RLock()

    def __deepcopy__(self, memo):
        import copy

        new = type(self).__new__(type(self))
        new.condition = self.condition
        new.combinables = [copy.deepcopy(c, memo) for c in self.combinables]
        new.data = []
        new._lock = threading.RLock()
        return new

    def check_and_send(self, collect):
        with self._lock:
            if self.condition(self.combinables):
                batch, self.data = self.data, []
                for c in self.combinables:
                    c.reset()
                if batch:  # an empty flush carries no message: nothing to route
                    collect(batch)

    def logic(self, func, collect):
        with self._lock:
            func(self.data)
            for c in self.combinables:
                c.logic(func, self.check_and_send, collect)

    def pending(self) -> int:
        with self._lock:
            return len(self.data)

    def flush(self, collect):
        with self._lock:
            if self.data:
                batch, self.data = self.data, []
                for c in self.combinables:
                    c.reset()
                collect(batch)

    def close(self):
        for c in self.combinables:
            c.close()


class CombinationWorkerSender(CombinationLogic, WorkerSender):
    def on_pull(self, param_id, collect, partition_id):
        self.logic(lambda buf: buf.append(WorkerToPS(partition_id, Left(Pull(param_id)))), collect)

    def on_push(self, param_id, delta, collect, partition_id):
        self.logic(lambda buf: buf.append(WorkerToPS(partition_id, Right(Push(param_id, delta)))), collect)


class CombinationPSSender(CombinationLogic, PSSender):
    def on_pull_answer(self, param_id, value, worker_partition_index, collect):
        self.logic(
            lambda buf: buf.append(PSToWorker(worker_partition_index, PullAnswer(param_id, value))), collect
        )


def wait_until(pred, timeout: float, interval: float = 0.01) -> bool:
    """Polling helper (ScalaTest ``Eventually`` analogue)."""
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if pred():
            return True
        time.sleep(interval)
    return pred()
