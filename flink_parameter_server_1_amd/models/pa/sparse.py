"""Sparse vectors for the Passive-Aggressive models.

``SparseVector`` plays Breeze's ``SparseVector[Double]`` (sorted unique
indices + values + length); ``VectorBuilder`` sums duplicate adds like
Breeze's builder.  ``HashSparseVector`` is the reference's own immutable
``HashMap[Long, E]`` vector with ``max_size`` and the ``EOFSign`` record
(``M/passive/aggressive/entities/SparseVector.scala:6-42``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, Tuple

import numpy as np


class SparseVector:
    __slots__ = ("indices", "values", "length")

    def __init__(self, indices, values, length: int):
        self.indices = np.asarray(indices, dtype=np.int64)
        self.values = np.asarray(values, dtype=np.float64)
        self.length = int(length)

    @staticmethod
    def from_pairs(pairs: Iterable[Tuple[int, float]], length: int) -> "SparseVector":
        b = VectorBuilder(length)
        for i, v in pairs:
            b.add(i, v)
        return b.to_sparse_vector()

    @property
    def active_size(self) -> int:
        return int(self.indices.size)

    def index_at(self, k):
        return int(self.indices[k])

    def value_at(self, k):
        return float(self.values[k])

    def norm_sq(self) -> float:
        return float(np.dot(self.values, self.values))

    def dot_dense(self, w: np.ndarray) -> float:
        return float(np.dot(self.values, w[self.indices]))

    def dot_map(self, m: Dict[int, float]) -> float:
        return float(sum(v * m.get(int(i), 0.0) for i, v in zip(self.indices, self.values)))

    def to_dense(self) -> np.ndarray:
        d = np.zeros(self.length)
        d[self.indices] = self.values
        return d

    def active_iterator(self):
        return zip(self.indices.tolist(), self.values.tolist())

    def __eq__(self, other):
        return (isinstance(other, SparseVector) and self.length == other.length
                and np.array_equal(self.indices, other.indices) and np.array_equal(self.values, other.values))

    def __hash__(self):
        return hash((self.length, self.indices.tobytes(), self.values.tobytes()))

    def __repr__(self):
        return f"SparseVector(len={self.length}, nnz={self.active_size})"


class VectorBuilder:
    def __init__(self, length: int):
        self.length = length
        self.idx = []
        self.val = []

    def add(self, i: int, v: float):
        self.idx.append(int(i))
        self.val.append(float(v))

    def to_sparse_vector(self) -> SparseVector:
        if not self.idx:
            return SparseVector([], [], self.length)
        idx = np.asarray(self.idx, dtype=np.int64)
        val = np.asarray(self.val, dtype=np.float64)
        uniq, inv = np.unique(idx, return_inverse=True)
        out = np.zeros(uniq.size)
        np.add.at(out, inv, val)
        return SparseVector(uniq, out, self.length)

    def to_dense_vector(self) -> np.ndarray:
        d = np.zeros(self.length)
        np.add.at(d, np.asarray(self.idx, dtype=np.int64), np.asarray(self.val))
        return d


@dataclass(frozen=True)
class HashSparseVector:
    """Immutable id -> value map with a logical ``max_size``."""

    max_size: int
    vector: Tuple[Tuple[int, float], ...]

    @staticmethod
    def build(max_size: int, items: Dict[int, float]) -> "HashSparseVector":
        return HashSparseVector(max_size, tuple(sorted(items.items())))

    def as_dict(self) -> Dict[int, float]:
        return dict(self.vector)


@dataclass(frozen=True)
class EOFSign:
    """End-of-stream marker of the offline PA apps (``SparseVector.scala:42``)."""

    worker_id: int
    minus_source_id: int
