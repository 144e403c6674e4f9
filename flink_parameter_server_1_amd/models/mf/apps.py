"""MF applications on the per-record engine (same entry points and defaults as the reference).

* ``ps_online_mf``  — ``PSOnlineMatrixFactorization.psOnlineMF``
  (``M/matrix/factorization/PSOnlineMatrixFactorization.scala:39-75``).  The
  reference passes ``negativeSampleRate``/``userMemory`` to the worker in
  swapped order; named arguments are used here.
* ``ps_offline_mf`` — ``PSOfflineMatrixFactorization.psOfflineMF``
  (``M/matrix/factorization/PSOfflineMatrixFactorization.scala:45-106``).
* ``ps_top_k_generator`` — ``PSTopKGenerator.psTopKGenerator``
  (``M/matrix/factorization/PSTopKGenerator.scala:47-107``): users on the PS
  (``Left`` model records), items worker-resident (``Right``), ratings
  broadcast to every worker, partial top-Ks merged at parallelism 1.
* ``ps_online_learner_and_generator`` —
  ``PSOnlineMatrixFactorizationAndTopKGenerator.psOnlineLearnerAndGenerator``
  (``M/matrix/factorization/PSOnlineMatrixFactorizationAndTopKGenerator.scala:50-100``).
* ``OnlineFactorModelBuilder`` — the abstract builder interface
  (``M/matrix/factorization/OnlineFactorModelBuilder.scala:5-12``).

Outputs follow the reference: ``Left((user, vec))`` from workers and
``Right((item, vec))`` from the PS for the MF apps; ``(user?, item, ts,
[(score, item)])`` tuples for the top-K apps.  For the GPU path of the same
model see ``models.mf.fast``.
"""
from __future__ import annotations

from typing import Iterable, Optional

from ...api.futures import BaseMFWorkerLogic
from ...api.limiters import add_pull_limiter
from ...core.engine import PartitionedInput, transform, transform_with_double_model_load
from ...core.messages import Left, Right
from ...ps.logics import SimplePSLogic
from ...utils.eof import with_eof
from .core import (USER_SEED_XOR, HashFactorInitializerDescriptor, IDGenerator, RangedRandomFactorInitializerDescriptor,
                   SGDUpdater, attach_length, vector_sum)
from .pruning import COORD, LI
from .workers import (CollectTopKFromEachWorker, PSOfflineMatrixFactorizationWorker,
                      PSOnlineMatrixFactorizationAndTopKGeneratorWorker, PSOnlineMatrixFactorizationWorker,
                      PSTopKGeneratorWorker)


def ps_online_mf(src: Iterable, num_factors: int = 10, range_min: float = -0.01, range_max: float = 0.01,
                 learning_rate: float = 0.01, negative_sample_rate: int = 0, user_memory: int = 128,
                 pull_limit: int = 1600, worker_parallelism: int = 4, ps_parallelism: int = 4,
                 iteration_wait_time: Optional[float] = None, seed: Optional[int] = None, runtime=None,
                 init: str = "ranged", lam: float = 0.0):
    """``init="hash"``: per-id hash init (items: seed, users: seed ^ USER_SEED_XOR), the
    init of ``ps_online_mf_native`` and the GPU tables (exact parity runs)."""
    user_init = None
    if init == "hash":
        init = HashFactorInitializerDescriptor(num_factors, range_min, range_max, seed or 0).open()
        user_init = HashFactorInitializerDescriptor(num_factors, range_min, range_max, (seed or 0) ^ USER_SEED_XOR)
    elif init == "ranged":
        init = RangedRandomFactorInitializerDescriptor(num_factors, range_min, range_max, seed).open()
    else:
        raise ValueError(f"init must be 'ranged' or 'hash', not {init!r}")
    worker = PSOnlineMatrixFactorizationWorker(num_factors, range_min, range_max, learning_rate,
                                               user_memory=user_memory, negative_sample_rate=negative_sample_rate,
                                               seed=seed, lam=lam, factor_init=user_init)
    ps_logic = SimplePSLogic(lambda i: init.next_factor(i), vector_sum)
    return transform(src, add_pull_limiter(worker, pull_limit), ps_logic,
                     worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism,
                     iteration_wait_time=iteration_wait_time, data_partitioner=lambda r: r.user, runtime=runtime)


def ps_offline_mf(src: Iterable, num_factors: int = 10, range_min: float = -0.01, range_max: float = 0.01,
                  learning_rate: float = 0.01, negative_sample_rate: int = 0, user_memory: int = 128,
                  iterations: int = 1, pull_limit: int = 1600, worker_parallelism: int = 4,
                  ps_parallelism: int = 4, iteration_wait_time: Optional[float] = None,
                  seed: Optional[int] = None, runtime=None):
    ratings = with_eof(src, worker_parallelism, partitioner=lambda r: r.user)
    worker = PSOfflineMatrixFactorizationWorker(num_factors, range_min, range_max, learning_rate,
                                                negative_sample_rate=negative_sample_rate, user_memory=user_memory,
                                                iterations=iterations, seed=seed)
    init = RangedRandomFactorInitializerDescriptor(num_factors, range_min, range_max, seed).open()
    return transform(ratings, add_pull_limiter(worker, pull_limit),
                     param_init=lambda i: init.next_factor(i), param_update=vector_sum,
                     worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism,
                     iteration_wait_time=iteration_wait_time, runtime=runtime)


def _broadcast(src, worker_parallelism):
    parts = [[] for _ in range(worker_parallelism)]
    for r in src:
        rid = IDGenerator.next()
        for i in range(worker_parallelism):
            parts[i].append(r.enrich(i, rid))
    return PartitionedInput(parts)


class _MFLimited(BaseMFWorkerLogic):
    """``BaseMFWorkerLogic.addPullLimiter``: pull limiter that forwards ``update_model``."""

    def __init__(self, inner, pull_limit):
        super().__init__()
        self.inner = inner
        self.lim = add_pull_limiter(inner, pull_limit)

    def open(self, ctx):
        self.lim.open(ctx)

    def on_recv(self, data, ps):
        self.lim.on_recv(data, ps)

    def on_pull_recv(self, pid, value, ps):
        self.lim.on_pull_recv(pid, value, ps)

    def update_model(self, pid, value):
        self.inner.update_model(pid, value)

    def close(self):
        self.lim.close()


def ps_top_k_generator(src: Iterable, model: Iterable, num_factors: int = 10, range_min: float = -0.01,
                       range_max: float = 0.01, user_memory: int = 0, K: int = 100, worker_k: int = 75,
                       bucket_size: int = 100, pruning_algorithm=COORD(), pull_limit: int = 1600,
                       worker_parallelism: int = 4, ps_parallelism: int = 4,
                       iteration_wait_time: Optional[float] = None, reference_quirks: bool = False, runtime=None):
    """``model``: ``Left((user, (len, vec)))`` -> PS, ``Right((item, (len, vec)))`` -> workers
    (items are dealt round-robin over workers like Flink's ``rebalance``).
    Returns ``(item, timestamp, top_k)`` per input rating."""
    invalid = (-1.0, [])
    worker = PSTopKGeneratorWorker(worker_k, bucket_size, worker_parallelism, pruning_algorithm, reference_quirks)
    ps_logic = SimplePSLogic(lambda _: invalid, lambda _, x: x)
    inputs = _broadcast(src, worker_parallelism)
    out = transform_with_double_model_load(model, inputs, _MFLimited(worker, pull_limit), ps_logic,
                                           worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism,
                                           iteration_wait_time=iteration_wait_time, runtime=runtime)
    merged = CollectTopKFromEachWorker(K, user_memory, worker_parallelism).run(out)
    return [(item, ts, topk) for (_, item, ts, topk) in merged]


def ps_online_learner_and_generator(src: Iterable, num_factors: int = 10, range_min: float = -0.001,
                                    range_max: float = 0.001, learning_rate: float = 0.01,
                                    negative_sample_rate: int = 0, user_memory: int = 65535, K: int = 100,
                                    worker_k: int = 75, bucket_size: int = 100, pruning_algorithm=LI(5, 2.5),
                                    pull_limit: int = 500, worker_parallelism: int = 4, ps_parallelism: int = 4,
                                    iteration_wait_time: Optional[float] = None, seed: Optional[int] = None,
                                    reference_quirks: bool = False, runtime=None, init: str = "ranged"):
    """``init="hash"``: per-id hash init (PS users: seed, worker items: seed ^
    USER_SEED_XOR) -- the init of the tensor-engine app, for exact parity runs."""
    if init == "hash":
        desc = HashFactorInitializerDescriptor(num_factors, range_min, range_max, ((seed or 0) ^ USER_SEED_XOR))
        ps_desc = HashFactorInitializerDescriptor(num_factors, range_min, range_max, seed or 0)
    elif init == "ranged":
        desc = ps_desc = RangedRandomFactorInitializerDescriptor(num_factors, range_min, range_max, seed)
    else:
        raise ValueError(f"init must be 'ranged' or 'hash', not {init!r}")
    worker = PSOnlineMatrixFactorizationAndTopKGeneratorWorker(
        negative_sample_rate=negative_sample_rate, user_memory=user_memory, worker_k=worker_k,
        bucket_size=bucket_size, pruning=pruning_algorithm, worker_parallelism=worker_parallelism,
        factor_init_desc=desc, factor_update=SGDUpdater(learning_rate), seed=seed,
        reference_quirks=reference_quirks)
    init = ps_desc.open() if ps_desc is not desc else desc.open()
    ps_logic = SimplePSLogic(lambda x: attach_length(init.next_factor(x)),
                             lambda vec, delta: attach_length(vector_sum(vec[1], delta[1])))
    out = transform(_broadcast(src, worker_parallelism), add_pull_limiter(worker, pull_limit), ps_logic,
                    worker_parallelism=worker_parallelism, ps_parallelism=ps_parallelism,
                    iteration_wait_time=iteration_wait_time, runtime=runtime)
    return CollectTopKFromEachWorker(K, user_memory, worker_parallelism).run(out)


class OnlineFactorModelBuilder:
    """Abstract ``buildModel(ratings, factorInit, factorUpdate, parameters)``."""

    def build_model(self, ratings, factor_init_desc, factor_update, parameters: dict):
        raise NotImplementedError

    buildModel = build_model


# Scala spelling
psOnlineMF = ps_online_mf
psOfflineMF = ps_offline_mf
psTopKGenerator = ps_top_k_generator
psOnlineLearnerAndGenerator = ps_online_learner_and_generator
