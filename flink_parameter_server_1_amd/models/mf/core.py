"""MF building blocks: vectors, ratings, factor initializers / updaters, top-K queues.

* vector math (``M/matrix/factorization/utils/Vector.scala``): ``vector_sum``
  raises ``FactorIsNotANumberException`` on NaN (``:72-84``);
  ``attach_length`` -> ``(|v|, v)``.
* ``Rating`` / ``RichRating`` (``M/matrix/factorization/utils/Rating.scala:9-31``).
* factor initializers (``M/matrix/factorization/factors/*``,
  ``M/matrix/factorization/PseudoRandomFactorInitializer.scala``).  The
  pseudo-random one is seeded with the id through a bit-exact port of
  ``java.util.Random`` so it reproduces the reference's values.
* ``SGDUpdater`` (``M/matrix/factorization/factors/SGDUpdater.scala``) with an
  optional L2 term (the reference's "fixme add lambda").
* ``TopKQueue`` — min-heap of ``(score, item)`` keeping the best ``k``
  (``M/matrix/factorization/utils/Utils.scala:23-30``).
"""
from __future__ import annotations

import heapq
import itertools
import random as _random
from dataclasses import dataclass
from typing import Callable, Iterable, List, Tuple

import numpy as np

Vector = np.ndarray
LengthAndVector = Tuple[float, np.ndarray]
UserId = int
ItemId = int


class FactorIsNotANumberException(ArithmeticError):
    pass


def vector_length_sqr(v) -> float:
    return float(np.dot(v, v))


def dot_product(u, v) -> float:
    return float(np.dot(u, v))


def vector_sum(u, v) -> np.ndarray:
    res = np.asarray(u, dtype=np.float64) + np.asarray(v, dtype=np.float64)
    if np.isnan(res).any():
        raise FactorIsNotANumberException()
    return res


def attach_length(u) -> LengthAndVector:
    u = np.asarray(u, dtype=np.float64)
    return (float(np.sqrt(vector_length_sqr(u))), u)


# ------------------------------------------------------------------ ratings
@dataclass(frozen=True)
class Rating:
    user: int
    item: int
    rating: float
    timestamp: int = 0

    def enrich(self, worker_id: int, rating_id: float) -> "RichRating":
        return RichRating(self.user, self.item, self.rating, worker_id, rating_id, self.timestamp)

    @staticmethod
    def from_tuple(t) -> "Rating":
        return Rating(int(t[0]), int(t[1]), float(t[2]), 0)

    fromTuple = from_tuple


@dataclass(frozen=True)
class RichRating:
    user: int
    item: int
    rating: float
    target_worker: int
    rating_id: float
    timestamp: int = 0

    def reduce(self) -> Rating:
        return Rating(self.user, self.item, self.rating, self.timestamp)


class IDGenerator:
    """Process-global monotonically increasing ids (``Utils.scala:39-46``)."""

    _counter = itertools.count()

    @classmethod
    def next(cls) -> int:
        return next(cls._counter)


# ------------------------------------------------------------------ java.util.Random
class JavaRandom:
    """Bit-exact ``java.util.Random`` (48-bit LCG) for reference parity."""

    _MUL, _ADD, _MASK = 0x5DEECE66D, 0xB, (1 << 48) - 1

    def __init__(self, seed: int):
        self.seed = (seed ^ self._MUL) & self._MASK

    def _next(self, bits: int) -> int:
        self.seed = (self.seed * self._MUL + self._ADD) & self._MASK
        r = self.seed >> (48 - bits)
        if bits == 32 and r >= 1 << 31:  # Java's (int) cast
            r -= 1 << 32
        return r

    def next_double(self) -> float:
        hi = self._next(26) & ((1 << 26) - 1)
        lo = self._next(27) & ((1 << 27) - 1)
        return ((hi << 27) + lo) * (1.0 / (1 << 53))

    def next_int(self, bound: int) -> int:
        if bound <= 0:
            raise ValueError("bound must be positive")
        if (bound & -bound) == bound:
            return ((bound * (self._next(31) & 0x7FFFFFFF)) >> 31)
        while True:
            bits = self._next(31) & 0x7FFFFFFF
            val = bits % bound
            if bits - val + (bound - 1) < (1 << 31):
                return val


# ------------------------------------------------------------------ initializers
class FactorInitializer:
    def next_factor(self, param_id: int) -> np.ndarray:
        raise NotImplementedError

    def nextFactor(self, param_id):  # noqa: N802
        return self.next_factor(param_id)


class FactorInitializerDescriptor:
    """Deferred construction (the reference defers non-serializable RNGs)."""

    def open(self) -> FactorInitializer:
        raise NotImplementedError

    @staticmethod
    def apply(init: Callable[[int], np.ndarray]) -> "FactorInitializerDescriptor":
        class _D(FactorInitializerDescriptor):
            def open(self_inner):
                class _I(FactorInitializer):
                    def next_factor(self, i):
                        return np.asarray(init(i), dtype=np.float64)

                return _I()

        return _D()


class RandomFactorInitializer(FactorInitializer):
    def __init__(self, rng: _random.Random, num_factors: int):
        self.rng, self.num_factors = rng, num_factors

    def next_factor(self, param_id):
        return np.array([self.rng.random() for _ in range(self.num_factors)])


@dataclass
class RandomFactorInitializerDescriptor(FactorInitializerDescriptor):
    num_factors: int
    seed: int = None

    def open(self):
        return RandomFactorInitializer(_random.Random(self.seed), self.num_factors)


class RangedRandomFactorInitializer(FactorInitializer):
    def __init__(self, rng, num_factors, range_min, range_max):
        self.rng, self.num_factors, self.lo, self.hi = rng, num_factors, range_min, range_max

    def next_factor(self, param_id):
        return np.array([self.lo + (self.hi - self.lo) * self.rng.random() for _ in range(self.num_factors)])


@dataclass
class RangedRandomFactorInitializerDescriptor(FactorInitializerDescriptor):
    num_factors: int
    range_min: float
    range_max: float
    seed: int = None

    def open(self):
        return RangedRandomFactorInitializer(_random.Random(self.seed), self.num_factors, self.range_min,
                                             self.range_max)


class PseudoRandomFactorInitializer(FactorInitializer):
    """``new Random(id)`` per id: deterministic, bit-identical to the reference."""

    def __init__(self, num_factors: int):
        self.num_factors = num_factors

    def next_factor(self, param_id):
        r = JavaRandom(int(param_id))
        return np.array([r.next_double() for _ in range(self.num_factors)])


@dataclass
class PseudoRandomFactorInitializerDescriptor(FactorInitializerDescriptor):
    num_factors: int

    def open(self):
        return PseudoRandomFactorInitializer(self.num_factors)


def _fmix32(x: int) -> int:
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & 0xFFFFFFFF
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & 0xFFFFFFFF
    return x ^ (x >> 16)


def hash_uniform01(seed: int, pid: int, j: int) -> float:
    """The stateless U[0,1) of the device tables and the native engines
    (``hash_uniform`` in csrc/kernels/common.h / csrc/host)."""
    h = _fmix32((seed ^ 0x9E3779B9) & 0xFFFFFFFF)
    h = _fmix32(h ^ (pid & 0xFFFFFFFF))
    h = _fmix32(h ^ ((pid >> 32) & 0xFFFFFFFF) ^ 0x27D4EB2F)
    h = _fmix32((h + j * 0x9E3779B9) & 0xFFFFFFFF)
    return (h >> 8) * (1.0 / 16777216.0)


class HashFactorInitializer(FactorInitializer):
    """U[lo, hi) per coordinate from a hash of (seed, id, coordinate): deterministic
    per id whatever the order of first touch (like ``PseudoRandomFactorInitializer``)
    and identical to the native record engine / GPU table init."""

    def __init__(self, num_factors, range_min, range_max, seed):
        self.num_factors, self.lo, self.hi, self.seed = num_factors, range_min, range_max, seed & 0xFFFFFFFF

    def next_factor(self, param_id):
        return np.array([self.lo + (self.hi - self.lo) * hash_uniform01(self.seed, int(param_id), j)
                         for j in range(self.num_factors)])


@dataclass
class HashFactorInitializerDescriptor(FactorInitializerDescriptor):
    num_factors: int
    range_min: float
    range_max: float
    seed: int = 0

    def open(self):
        return HashFactorInitializer(self.num_factors, self.range_min, self.range_max, self.seed)


#: seed offset of the user-side hash init (the item side uses the job seed)
USER_SEED_XOR = 0x5BD1E995


# ------------------------------------------------------------------ updaters
class FactorUpdater:
    def delta(self, rating: float, user, item) -> Tuple[np.ndarray, np.ndarray]:
        raise NotImplementedError


class SGDUpdater(FactorUpdater):
    """``e = r - u.i``; ``(lr*e*i - lr*lam*u, lr*e*u - lr*lam*i)``."""

    def __init__(self, learning_rate: float, lam: float = 0.0):
        self.learning_rate = learning_rate
        self.lam = lam

    def delta(self, rating, user, item):
        user = np.asarray(user, dtype=np.float64)
        item = np.asarray(item, dtype=np.float64)
        e = rating - float(np.dot(user, item))
        lr = self.learning_rate
        if self.lam:
            return lr * (e * item - self.lam * user), lr * (e * user - self.lam * item)
        return lr * e * item, lr * e * user


# ------------------------------------------------------------------ top-K
class TopKQueue:
    """Min-heap of ``(score, item)``; ``head`` is the smallest kept score."""

    def __init__(self, items: Iterable[Tuple[float, int]] = ()):
        self._h: List[Tuple[float, int]] = list(items)
        heapq.heapify(self._h)

    def __len__(self):
        return len(self._h)

    def push(self, score: float, item: int):
        heapq.heappush(self._h, (score, item))

    def offer(self, score: float, item: int, k: int):
        """Keep the best ``k``: the reference's ``size<k ? add : replace-min-if-better``."""
        if len(self._h) < k:
            heapq.heappush(self._h, (score, item))
        elif self._h[0][0] < score:
            heapq.heapreplace(self._h, (score, item))

    @property
    def head(self) -> Tuple[float, int]:
        return self._h[0]

    def items(self) -> List[Tuple[float, int]]:
        return list(self._h)

    def sorted_desc(self) -> List[Tuple[float, int]]:
        return sorted(self._h, key=lambda x: (-x[0], x[1]))

    def __iter__(self):
        return iter(self._h)


def new_top_k_queue() -> TopKQueue:
    return TopKQueue()
