"""Offline (multi-epoch) Passive-Aggressive classification apps + the legacy PA filter.

* ``PassiveAggressiveFilter`` (``M/passive/aggressive/algorithm/binary/PassiveAggressiveFilter.scala:7-49``):
  binary PA on ``{feature: weight}`` maps with labels +-1.  The reference's
  PA-II uses integer division ``1 / (2 * C)`` (0 for C >= 1); the
  float form is used here.  ``MulticlassPassiveAggressiveFilter`` is the OVA
  counterpart the reference only declares (``.../multi/PassiveAggressiveFilter.scala``).
* ``pa_binary_classification_offline`` — ``PABinaryClassificationOffline``
  (``M/passive/aggressive/classification/binary/PABinaryClassificationOffline.scala:47-387``):
  workers buffer training and test data until end of input, run
  ``iterations`` shuffled epochs of pull -> delta -> push (the reference's
  no-op shuffle, B2, is fixed), wait until every training answer has been
  applied, then pull the test vectors' weights and predict.  Predictions are
  emitted as worker outputs and logged at close in the reference's
  ``###PS###t;<label>;[k -> v,...]`` format.
* ``pa_multi_classification_offline`` — the multiclass app.  The reference's
  ``PAMultiClassificationOffline`` is a byte copy of the binary one (B8); this
  one really is multiclass (OVA filter, integer labels).
"""
from __future__ import annotations

import logging
import random
from collections import defaultdict, deque
from typing import Dict, Iterable, List, Optional

import numpy as np

from ...api.limiters import add_pull_limiter
from ...api.logic import WorkerLogic
from ...core.engine import PartitionedInput, split_input, transform
from ...ps.logics import SimplePSLogic
from .algorithms import RandomModelInitializer

log = logging.getLogger("flink_parameter_server_1_amd.pa.offline")


class PassiveAggressiveFilter:
    def __init__(self, c: float = 0.0):
        self.const = float(c)

    def get_tau(self, norm_sq: float, loss: float) -> float:
        raise NotImplementedError

    @staticmethod
    def _quotient(norm_sq, loss, denominator_const):
        den = norm_sq + denominator_const
        return loss / den if den else 0.0

    def delta(self, data: Dict[int, float], model: Dict[int, float], label: int):
        if label not in (1, -1):
            raise ValueError("binary labels are +1 / -1")
        if set(data) != set(model):
            raise ValueError("model must hold exactly the data's features")
        margin = sum(model[k] * v for k, v in data.items())
        loss = max(0.0, 1.0 - label * margin)
        mult = self.get_tau(sum(v * v for v in data.values()), loss) * label
        return {k: v * mult for k, v in data.items()}

    def predict(self, data, model) -> int:
        return int(np.sign(sum(model[k] * v for k, v in data.items())))

    @staticmethod
    def build_paf():
        return _PAF()

    @staticmethod
    def build_pafi(c):
        return _PAFI(c)

    @staticmethod
    def build_pafii(c):
        return _PAFII(c)

    buildPAF, buildPAFI, buildPAFII = build_paf, build_pafi, build_pafii


class _PAF(PassiveAggressiveFilter):
    def get_tau(self, n, loss):
        return self._quotient(n, loss, 0.0)


class _PAFI(PassiveAggressiveFilter):
    def get_tau(self, n, loss):
        return min(self.const, self._quotient(n, loss, 0.0))


class _PAFII(PassiveAggressiveFilter):
    def get_tau(self, n, loss):
        return self._quotient(n, loss, 1.0 / (2.0 * self.const))


class MulticlassPassiveAggressiveFilter:
    """OVA filter on ``{feature: L-vector}`` maps, integer labels."""

    def __init__(self, label_count: int, paf_type: int = 0, c: float = 0.0):
        self.L, self.type, self.const = label_count, paf_type, float(c)

    def _tau(self, n, loss):
        if self.type == 0:
            return loss / n if n else np.zeros_like(loss)
        if self.type == 1:
            return np.minimum(self.const, loss / n) if n else np.zeros_like(loss)
        return loss / (n + 1.0 / (2.0 * self.const))

    def delta(self, data, model, label: int):
        y = -np.ones(self.L)
        y[label] = 1.0
        d = sum(v * np.asarray(model[k]) for k, v in data.items())
        loss = np.maximum(0.0, 1.0 - d * y)
        mult = self._tau(sum(v * v for v in data.values()), loss) * y
        return {k: v * mult for k, v in data.items()}

    def predict(self, data, model) -> int:
        return int(np.argmax(sum(v * np.asarray(model[k]) for k, v in data.items())))


def build_filter(paf_type: int, paf_const: float):
    if paf_type == 0:
        return PassiveAggressiveFilter.build_paf()
    if paf_type == 1:
        return PassiveAggressiveFilter.build_pafi(paf_const)
    if paf_type == 2:
        return PassiveAggressiveFilter.build_pafii(paf_const)
    raise ValueError("PassiveAggressiveFilter type can be only in the set (0, 1, 2)")


class _OfflineWorker(WorkerLogic):
    """Buffers train/test data until EOF, trains ``iterations`` epochs, then predicts."""

    def __init__(self, paf, iterations: int, seed: Optional[int] = None):
        self.paf = paf
        self.iterations = iterations
        self.train: List[tuple] = []
        self.test: List[dict] = []
        self.waiting: Dict[int, deque] = defaultdict(deque)
        self.outstanding = 0
        self.predicting = False
        self.predictions: List[tuple] = []
        self.rng = random.Random(seed)
        self.ps = None

    def on_recv(self, rec, ps):
        kind, payload = rec
        if kind == "train":
            self.train.append(payload)
        elif kind == "test":
            self.test.append(payload)
        else:  # EOF: all epochs' pulls (the limiter releases them as answers arrive)
            self.ps = ps
            if not self.train:
                self._start_prediction(ps)
                return
            for _ in range(self.iterations):
                order = list(range(len(self.train)))
                self.rng.shuffle(order)
                for i in order:
                    self._pull_example(("train", i), self.train[i][0], ps)

    def _pull_example(self, tag, data, ps):
        buf = {}
        self.outstanding += 1
        for k in data:
            self.waiting[k].append((tag, buf, len(data)))
            ps.pull(k)

    def _start_prediction(self, ps):
        self.predicting = True
        for j, vec in enumerate(self.test):
            self._pull_example(("test", j), vec, ps)

    def on_pull_recv(self, pid, value, ps):
        q = self.waiting[pid]
        tag, buf, need = q.popleft()
        if not q:
            del self.waiting[pid]
        buf[pid] = value
        if len(buf) < need:
            return
        self.outstanding -= 1
        kind, i = tag
        if kind == "train":
            vec, label = self.train[i]
            for k, v in self.paf.delta(vec, buf, label).items():
                ps.push(k, v)
            if self.outstanding == 0 and not self.predicting:
                self._start_prediction(ps)
        else:
            vec = self.test[i]
            label = self.paf.predict(vec, buf)
            self.predictions.append((vec, label))
            ps.output((vec, label))

    def close(self):
        for vec, label in self.predictions:
            log.info("###PS###t;%s;[%s]", label, ",".join(f"{k} -> {v}" for k, v in sorted(vec.items())))


def _offline_inputs(training: Iterable, test: Iterable, W: int) -> PartitionedInput:
    tr = split_input([("train", x) for x in training], W)
    te = split_input([("test", x) for x in test], W)
    return PartitionedInput([list(a) + list(b) + [("eof", None)] for a, b in zip(tr, te)])


def pa_binary_classification_offline(training: Iterable, test: Iterable, worker_parallelism: int,
                                     ps_parallelism: int, iterations: int, paf_type: int, paf_const: float,
                                     pull_limit: int, iteration_wait_time=None, seed: Optional[int] = None,
                                     runtime=None):
    """``training``: ``(features: {id: value}, label in {+1, -1})``; ``test``: ``{id: value}``.
    Outputs ``Left((test_vector, predicted_label))`` and ``Right((feature, weight))`` per push."""
    worker = add_pull_limiter(_OfflineWorker(build_filter(paf_type, paf_const), iterations, seed), pull_limit)
    server = SimplePSLogic(lambda _: RandomModelInitializer.init(), lambda a, b: a + b)
    return transform(_offline_inputs(training, test, worker_parallelism), worker, server,
                     param_partitioner=lambda m: abs(m.msg.value.param_id) % ps_parallelism,
                     worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism,
                     iteration_wait_time=iteration_wait_time, runtime=runtime)


def pa_multi_classification_offline(training: Iterable, test: Iterable, label_count: int, worker_parallelism: int,
                                    ps_parallelism: int, iterations: int, paf_type: int, paf_const: float,
                                    pull_limit: int, iteration_wait_time=None, seed: Optional[int] = None,
                                    runtime=None):
    """Multiclass counterpart: labels ``0..label_count-1``; weights are L-vectors."""
    worker = add_pull_limiter(
        _OfflineWorker(MulticlassPassiveAggressiveFilter(label_count, paf_type, paf_const), iterations, seed),
        pull_limit)
    server = SimplePSLogic(lambda _: np.zeros(label_count), lambda a, b: a + b)
    return transform(_offline_inputs(training, test, worker_parallelism), worker, server,
                     param_partitioner=lambda m: abs(m.msg.value.param_id) % ps_parallelism,
                     worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism,
                     iteration_wait_time=iteration_wait_time, runtime=runtime)


paBinaryClassificationOffline = pa_binary_classification_offline
paMultiClassificationOffline = pa_multi_classification_offline
