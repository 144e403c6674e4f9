"""Passive-Aggressive learners (Crammer et al. 2006) — the reference's L6 math.

* binary PA / PA-I / PA-II (``M/passive/aggressive/algorithm/PassiveAggressiveBinaryAlgorithm.scala``):
  ``loss = max(0, 1 - y (x.w))``; ``tau = loss/|x|^2`` | ``min(C, loss/|x|^2)`` |
  ``loss/(|x|^2 + 1/(2C))``; ``delta_i = tau*y*x_i`` on the active features.
* multiclass one-vs-all (``.../PassiveAggressiveOneVersusAll.scala``):
  ``y in {+-1}^L``, ``d = W^T x``, per-class loss/tau, ``delta_i = x_i (tau * y)``.
* cost-sensitive prediction-based / max-loss (``.../PassiveAggressiveCostBased.scala``):
  ``loss = d_q - d_y + sqrt(cost(y, q))``, ``tau = loss / (2 |x|^2)``; PB takes
  ``q = argmax d``, ML ``q = argmax(d_i - d_y + sqrt(cost(y,i)))``; if ``q != y``
  every active feature gets ``{y: tau x_i, q: -tau x_i}``.  The reference's
  builder is shared and never cleared so deltas accumulate across features and
  calls; each delta here is independent.

``model`` arguments are the parameters gathered for the example's active
features only: a ``{feature: value}`` dict (binary) or ``{feature: L-vector}``
dict (multiclass) -- what the worker assembled from its pull answers.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Tuple

import numpy as np

from .sparse import SparseVector


class PassiveAggressiveAlgorithm:
    def delta(self, x: SparseVector, model, label) -> List[Tuple[int, object]]:
        raise NotImplementedError

    def predict(self, x: SparseVector, model):
        raise NotImplementedError


# ---------------------------------------------------------------- binary
class PassiveAggressiveBinaryAlgorithm(PassiveAggressiveAlgorithm):
    variant = "PA"

    def __init__(self, aggressiveness: float = 0.0):
        self.aggressiveness = float(aggressiveness)

    def tau(self, norm_sq: float, loss: float) -> float:
        raise NotImplementedError

    @staticmethod
    def margin(x: SparseVector, model) -> float:
        if isinstance(model, dict):
            return x.dot_map(model)
        return x.dot_dense(np.asarray(model))

    def delta(self, x, model, label: bool):
        y = 1.0 if label else -1.0
        loss = max(0.0, 1.0 - y * self.margin(x, model))
        mult = self.tau(x.norm_sq(), loss) * y
        if mult == 0.0:
            return []
        return list(zip(x.indices.tolist(), (x.values * mult).tolist()))

    def predict(self, x, model) -> bool:
        return self.margin(x, model) > 0

    @staticmethod
    def build_pa():
        return _BinPA()

    @staticmethod
    def build_pai(c: float):
        return _BinPAI(c)

    @staticmethod
    def build_paii(c: float):
        return _BinPAII(c)

    buildPA, buildPAI, buildPAII = build_pa, build_pai, build_paii


def _quotient(norm_sq, loss, denominator_const):
    if norm_sq == 0.0 and denominator_const == 0:
        return 0.0
    return loss / (norm_sq + denominator_const)


class _BinPA(PassiveAggressiveBinaryAlgorithm):
    variant = "PA"

    def tau(self, n, loss):
        return _quotient(n, loss, 0.0)


class _BinPAI(PassiveAggressiveBinaryAlgorithm):
    variant = "PA-I"

    def tau(self, n, loss):
        return min(self.aggressiveness, _quotient(n, loss, 0.0))


class _BinPAII(PassiveAggressiveBinaryAlgorithm):
    variant = "PA-II"

    def tau(self, n, loss):
        return _quotient(n, loss, 1.0 / (2.0 * self.aggressiveness))


# ---------------------------------------------------------------- multiclass
class PassiveAggressiveMulticlassAlgorithm(PassiveAggressiveAlgorithm):
    def __init__(self, label_count: int):
        self.label_count = label_count

    def decision(self, x: SparseVector, model: Dict[int, np.ndarray]) -> np.ndarray:
        d = np.zeros(self.label_count)
        for i, v in x.active_iterator():
            w = model.get(i)
            if w is not None:
                d += v * np.asarray(w)
        return d

    def predict(self, x, model) -> int:
        if isinstance(model, np.ndarray):  # dense [features, L]
            return int(np.argmax(x.values @ model[x.indices]))
        return int(np.argmax(self.decision(x, model)))

    def delta(self, x, model, label: int):
        return self.delta_mtx(x, model, label)


class PassiveAggressiveOneVersusAll(PassiveAggressiveMulticlassAlgorithm):
    variant = "PA"

    def __init__(self, label_count: int, aggressiveness: float = 0.0):
        super().__init__(label_count)
        self.aggressiveness = float(aggressiveness)

    @staticmethod
    def loss(decision: np.ndarray, label_vec: np.ndarray) -> np.ndarray:
        return np.maximum(0.0, 1.0 - decision * label_vec)

    def tau(self, norm_sq: float, loss: np.ndarray) -> np.ndarray:
        raise NotImplementedError

    def delta_mtx(self, x, model, label: int):
        y = -np.ones(self.label_count)
        y[label] = 1.0
        mult = self.tau(x.norm_sq(), self.loss(self.decision(x, model), y)) * y
        if not mult.any():
            return []
        return [(i, v * mult) for i, v in x.active_iterator()]

    @staticmethod
    def build_pa(label_count: int):
        return _OvaPA(label_count)

    @staticmethod
    def build_pai(label_count: int, c: float):
        return _OvaPAI(label_count, c)

    @staticmethod
    def build_paii(label_count: int, c: float):
        return _OvaPAII(label_count, c)

    buildPA, buildPAI, buildPAII = build_pa, build_pai, build_paii


class _OvaPA(PassiveAggressiveOneVersusAll):
    def tau(self, n, loss):
        return loss / n if n else np.zeros_like(loss)


class _OvaPAI(PassiveAggressiveOneVersusAll):
    variant = "PA-I"

    def tau(self, n, loss):
        return np.minimum(self.aggressiveness, loss / n) if n else np.zeros_like(loss)


class _OvaPAII(PassiveAggressiveOneVersusAll):
    variant = "PA-II"

    def tau(self, n, loss):
        return loss / (n + 1.0 / (2.0 * self.aggressiveness))


class PassiveAggressiveCostBased(PassiveAggressiveMulticlassAlgorithm):
    variant = "PB"

    def __init__(self, cost: Callable[[int, int], float], label_count: int):
        super().__init__(label_count)
        self.cost = cost

    def loss(self, d, q, label) -> float:
        return d[q] - d[label] + math.sqrt(self.cost(label, q))

    @staticmethod
    def tau(x: SparseVector, loss: float) -> float:
        n = x.norm_sq()
        return loss / (2.0 * n) if n else 0.0

    def quotient(self, d: np.ndarray, label: int) -> int:
        raise NotImplementedError

    def delta_mtx(self, x, model, label: int):
        d = self.decision(x, model)
        q = self.quotient(d, label)
        if q == label:
            return []
        t = self.tau(x, self.loss(d, q, label))
        out = []
        for i, v in x.active_iterator():
            vec = np.zeros(self.label_count)
            vec[label] += t * v
            vec[q] -= t * v
            out.append((i, vec))
        return out

    @staticmethod
    def build_pb(cost, label_count):
        return _CostPB(cost, label_count)

    @staticmethod
    def build_ml(cost, label_count):
        return _CostML(cost, label_count)

    buildPB, buildML = build_pb, build_ml


class _CostPB(PassiveAggressiveCostBased):
    variant = "PB"

    def quotient(self, d, label):
        return int(np.argmax(d))


class _CostML(PassiveAggressiveCostBased):
    variant = "ML"

    def quotient(self, d, label):
        costs = np.array([math.sqrt(self.cost(label, i)) for i in range(self.label_count)])
        return int(np.argmax(d - d[label] + costs))


# ---------------------------------------------------------------- initializers
def init_binary(_: int) -> float:
    """``PassiveAggressiveParameterInitializer.initBinary`` (zeros)."""
    return 0.0


def init_multi(label_count: int):
    return lambda _: np.zeros(label_count)


class RandomModelInitializer:
    """``RandomModelInitializer.init() = 0`` (``M/passive/aggressive/algorithm/RandomModelInitializer.scala``)."""

    @staticmethod
    def init() -> float:
        return 0.0
