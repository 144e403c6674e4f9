"""Native per-record engine for ``psOnlineMF`` on CPU (BASELINE config #1).

``ps_online_mf_native`` runs the reference's online MF job -- W worker and P PS
subtasks exchanging one pull, one pull answer and one push per rating through
FIFO mailboxes, pull limiter, per-item rating FIFOs, lazy init, add-merging PS
-- in C++ (``csrc/host/record_engine.cpp``), with the scheduling turn of
``core.engine.LocalRuntime``.  Same semantics as
``models.mf.apps.ps_online_mf(..., init="hash")`` (tested equal on the folded
model); the Python engine remains the one that runs arbitrary user
``WorkerLogic`` / ``ParameterServerLogic`` callbacks.

Reference: ``M/matrix/factorization/PSOnlineMatrixFactorization.scala:39-75``,
``M/matrix/factorization/workers/PSOnlineMatrixFactorizationWorker.scala:22-90``,
``M/server/SimplePSLogic.scala:7-26``, ``M/WorkerLogic.scala:176-225``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict

import numpy as np

from ...utils import native_host
from .core import FactorIsNotANumberException


@dataclass
class NativeMFResult:
    user_ids: np.ndarray      # int64 [U]
    user_vectors: np.ndarray  # float64 [U, D]
    item_ids: np.ndarray      # int64 [I]
    item_vectors: np.ndarray  # float64 [I, D]
    stats: Dict[str, int]

    def users(self) -> Dict[int, np.ndarray]:
        return {int(i): v for i, v in zip(self.user_ids, self.user_vectors)}

    def items(self) -> Dict[int, np.ndarray]:
        return {int(i): v for i, v in zip(self.item_ids, self.item_vectors)}


_STATS = ("pulls", "pushes", "answers", "worker_outputs", "ps_outputs", "turns", "negatives")


def ps_online_mf_native(users, items, ratings, num_factors: int = 10, range_min: float = -0.01,
                        range_max: float = 0.01, learning_rate: float = 0.01, lam: float = 0.0,
                        negative_sample_rate: int = 0, user_memory: int = 128, pull_limit: int = 1600,
                        worker_parallelism: int = 4, ps_parallelism: int = 4, seed: int = 0) -> NativeMFResult:
    """Online MF over the rating stream ``(users[k], items[k], ratings[k])`` in order."""
    L = native_host.lib()
    if L is None:
        raise RuntimeError("host library unavailable: run python csrc/build.py --only host")
    u = np.ascontiguousarray(users, dtype=np.int64)
    it = np.ascontiguousarray(items, dtype=np.int64)
    r = np.ascontiguousarray(ratings, dtype=np.float64)
    n = u.shape[0]
    if it.shape[0] != n or r.shape[0] != n:
        raise ValueError("users, items and ratings need the same length")
    D = int(num_factors)
    n_users = int(np.unique(u).size) if n else 0
    n_items = int(np.unique(it).size) if n else 0
    uid = np.empty(max(n_users, 1), dtype=np.int64)
    uval = np.empty((max(n_users, 1), D), dtype=np.float64)
    iid = np.empty(max(n_items, 1), dtype=np.int64)
    ival = np.empty((max(n_items, 1), D), dtype=np.float64)
    counts = np.zeros(2, dtype=np.int64)
    stats = np.zeros(len(_STATS), dtype=np.int64)
    p = native_host._p
    rc = L.fps_mf_online_record(p(u), p(it), p(r), n, int(worker_parallelism), int(ps_parallelism), D,
                                float(learning_rate), float(lam), float(range_min), float(range_max),
                                int(seed) & 0xFFFFFFFF, int(pull_limit), int(negative_sample_rate), int(user_memory),
                                p(uid), p(uval), uid.shape[0], p(iid), p(ival), iid.shape[0], p(counts), p(stats))
    if rc == -1:
        raise FactorIsNotANumberException()
    if rc != 0:
        raise RuntimeError(f"fps_mf_online_record failed ({rc})")
    nu, ni = int(counts[0]), int(counts[1])
    return NativeMFResult(uid[:nu].copy(), uval[:nu].copy(), iid[:ni].copy(), ival[:ni].copy(),
                          dict(zip(_STATS, map(int, stats))))


__all__ = ["ps_online_mf_native", "NativeMFResult"]
