"""Passive-Aggressive on the parameter server (per-record engine).

``transform_binary`` / ``transform_multiclass`` / ``transform_multiclass_with_long_id``
mirror ``PassiveAggressiveParameterServer`` (``M/passive/aggressive/PassiveAggressiveParameterServer.scala``):

* input records: ``Left((vector, label))`` labelled (train) or
  ``Right((id, vector))`` unlabelled (predict)  (``:27-31``);
* the worker pulls **every active feature** of an example (``:289-307``),
  collects the answers in a per-example buffer and, when all arrived, builds
  the local model; labelled -> push per-feature deltas, unlabelled -> output
  ``(id or vector, predicted label)`` (``:309-336``);
* PS: ``RangePSLogicWithClose`` with range partitioning or
  ``SimplePSLogicWithClose`` with ``|id| % P`` (``:262-281``); the model is
  dumped as ``Right((feature, param))`` at close; optional warm start through
  ``transform_with_model_load`` (``:345-354``);
* the worker is wrapped in a pull limiter (``:283``).

The tensor/GPU version (batched, HIP kernels) is ``models.pa.fast``.
"""
from __future__ import annotations

from collections import defaultdict, deque
from typing import Iterable, Optional

import numpy as np

from ...api.limiters import add_pull_limiter
from ...api.logic import WorkerLogic
from ...core.engine import transform, transform_with_model_load
from ...core.partitioners import range_partitioner_ps
from ...ps.logics import RangePSLogicWithClose, SimplePSLogicWithClose
from .algorithms import init_binary, init_multi


class _PAWorker(WorkerLogic):
    """Pull all active features, train or predict when the last answer arrives."""

    def __init__(self, method, id_of):
        self.method = method
        self.id_of = id_of
        self.waiting = defaultdict(deque)

    def on_recv(self, data, ps):
        vec = data.value[0] if data.is_left else data.value[1]
        buf = {}
        for k in vec.indices.tolist():
            self.waiting[k].append((data, buf))
            ps.pull(k)

    def on_pull_recv(self, param_id, value, ps):
        q = self.waiting[param_id]
        data, buf = q.popleft()
        if not q:
            del self.waiting[param_id]
        buf[param_id] = value
        vec = data.value[0] if data.is_left else data.value[1]
        if len(buf) == vec.active_size:
            if data.is_left:
                for i, d in self.method.delta(vec, buf, data.value[1]):
                    ps.push(i, d)
            else:
                ps.output((self.id_of(data), self.method.predict(vec, buf)))


def _add(a, b):
    return a + b


def transform_generic(model: Optional[Iterable], init, input_source, worker_parallelism: int, ps_parallelism: int,
                      method, pull_limit: int, feature_count: int, range_partitioning: bool,
                      iteration_wait_time=None, id_of=None, runtime=None):
    if range_partitioning:
        server = RangePSLogicWithClose(feature_count, init, _add)
        partitioner = range_partitioner_ps(feature_count)(ps_parallelism)
    else:
        server = SimplePSLogicWithClose(init, _add)
        partitioner = lambda m: abs(m.msg.value.param_id) % ps_parallelism  # noqa: E731
    worker = add_pull_limiter(_PAWorker(method, id_of or (lambda d: d.value[1])), pull_limit)
    w_in = lambda m: m.worker_partition_index  # noqa: E731
    if model is not None:
        return transform_with_model_load(model, input_source, worker, server, param_partitioner=partitioner,
                                         w_in_partition=w_in, worker_parallelism=worker_parallelism,
                                         ps_parallelism=ps_parallelism, iteration_wait_time=iteration_wait_time,
                                         runtime=runtime)
    return transform(input_source, worker, server, param_partitioner=partitioner, w_in_partition=w_in,
                     worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism,
                     iteration_wait_time=iteration_wait_time, runtime=runtime)


def transform_binary(model: Optional[Iterable] = None, *, input_source, worker_parallelism: int,
                     ps_parallelism: int, passive_aggressive_method, pull_limit: int, feature_count: int,
                     range_partitioning: bool, iteration_wait_time=None, runtime=None):
    """Binary PA; predictions are ``Left((vector, bool))``, model ``Right((feature, weight))``."""
    return transform_generic(model, init_binary, input_source, worker_parallelism, ps_parallelism,
                             passive_aggressive_method, pull_limit, feature_count, range_partitioning,
                             iteration_wait_time, id_of=lambda d: d.value[1], runtime=runtime)


def transform_multiclass(model: Optional[Iterable] = None, *, input_source, worker_parallelism: int,
                         ps_parallelism: int, passive_aggressive_method, pull_limit: int, label_count: int,
                         feature_count: int, range_partitioning: bool, iteration_wait_time=None, runtime=None):
    """Multiclass PA (OVA / cost-based); predictions ``Left((vector, class))``."""
    return transform_generic(model, init_multi(label_count), input_source, worker_parallelism, ps_parallelism,
                             passive_aggressive_method, pull_limit, feature_count, range_partitioning,
                             iteration_wait_time, id_of=lambda d: d.value[1], runtime=runtime)


def transform_multiclass_with_long_id(model: Optional[Iterable] = None, *, input_source, worker_parallelism: int,
                                      ps_parallelism: int, passive_aggressive_method, pull_limit: int,
                                      label_count: int, feature_count: int, range_partitioning: bool,
                                      iteration_wait_time=None, runtime=None):
    """Multiclass PA where unlabelled inputs carry a ``long`` id: predictions ``Left((id, class))``."""
    return transform_generic(model, init_multi(label_count), input_source, worker_parallelism, ps_parallelism,
                             passive_aggressive_method, pull_limit, feature_count, range_partitioning,
                             iteration_wait_time, id_of=lambda d: d.value[0], runtime=runtime)


def binary_accuracy(model_weights: np.ndarray, labelled, method) -> float:
    """``PassiveAggressiveBinaryModelEvaluation.accuracy`` (percent correct), with the
    confusion counts (``T/test/utils/PassiveAggressiveBinaryModelEvaluation.scala:14-41``)."""
    tt = ff = tf = ft = 0
    for vec, lab in labelled:
        if lab is None:
            raise ValueError("Labels should not be missing.")
        pred = method.predict(vec, model_weights)
        if lab and pred:
            tt += 1
        elif not lab and not pred:
            ff += 1
        elif lab:
            tf += 1
        else:
            ft += 1
    n = tt + ff + tf + ft
    return 100.0 * (tt + ff) / max(n, 1)


def multi_accuracy(model_matrix: np.ndarray, labelled, method) -> float:
    """``PassiveAggressiveMultiModelEvaluation.accuracy`` (percent correct)."""
    ok = sum(int(method.predict(vec, model_matrix) == lab) for vec, lab in labelled)
    return 100.0 * ok / max(len(labelled), 1)


# Scala spelling
transformBinary = transform_binary
transformMulticlass = transform_multiclass
transformMulticlassWithLongId = transform_multiclass_with_long_id
