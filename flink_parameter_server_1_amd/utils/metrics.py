"""Quality evaluators and runtime metrics.

Evaluators (test-side in the reference, library utilities here):
* ``rmse`` — ``PSOfflineMatrixFactorizationTest.computeRMSE`` (``T/.../PSOfflineMatrixFactorizationTest.scala:36-47``);
* ``ndcg_at_k`` / ``NDCGAggregator`` — ``nDCGSink``: nDCG@K = ``log 2 / log(1 + rank)``
  if the true item is in the top-K else 0, aggregated per period
  ``timestamp // period`` with hit counts (``T/.../sink/nDCGSink.scala:192-272``);
  CSV / text writers like ``nDCGToCsv`` / ``nDCGPeriodsToCsv``;
* ``recall_precision_at_k`` — the notebooks' top-5 evaluation (``Notebooks/Tester.ipynb``).

Runtime metrics (the reference has none): ``Counters`` (per-rank pulls,
pushes, unique keys, bytes sent), ``StageTimer`` (HIP-event or wall timed
stages), JSON-lines output and the headline updates/s.
"""
from __future__ import annotations

import json
import math
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np


def rmse(ratings, users: Dict[int, np.ndarray], items: Dict[int, np.ndarray]) -> float:
    s = 0.0
    n = 0
    for r in ratings:
        d = float(np.dot(users[r.user], items[r.item])) - r.rating
        s += d * d
        n += 1
    return math.sqrt(s / max(n, 1))


def ndcg_at_k(top_k: Sequence[int], true_item: int) -> float:
    for rank, item in enumerate(top_k, start=1):
        if item == true_item:
            return math.log(2.0) / math.log(1.0 + rank)
    return 0.0


class NDCGAggregator:
    """Per-period nDCG and hit-rate of top-K recommendations (``nDCGSink``)."""

    def __init__(self, period_length: int = 86400):
        self.period_length = period_length
        self.sum = defaultdict(float)
        self.hits = defaultdict(int)
        self.count = defaultdict(int)

    def add(self, timestamp: int, top_k: Sequence, true_item: int):
        items = [x[1] if isinstance(x, tuple) else x for x in top_k]
        p = int(timestamp) // self.period_length
        v = ndcg_at_k(items, true_item)
        self.sum[p] += v
        self.hits[p] += int(v > 0)
        self.count[p] += 1

    def add_stream(self, records: Iterable[Tuple]):
        """Records ``(user, item, timestamp, [(score, item)...])`` as produced by the top-K apps."""
        for rec in records:
            _, item, ts, topk = rec[-4:] if len(rec) >= 4 else (None,) + tuple(rec)
            self.add(ts, topk, item)

    def periods(self) -> List[Tuple[int, float, float, int]]:
        """``(period, mean nDCG, hit rate, count)`` sorted by period."""
        return [(p, self.sum[p] / self.count[p], self.hits[p] / self.count[p], self.count[p])
                for p in sorted(self.count)]

    def to_csv(self, path: str):
        with open(path, "w") as f:
            f.write("period,ndcg,hit_rate,count\n")
            for p, nd, hr, c in self.periods():
                f.write(f"{p},{nd:.6f},{hr:.6f},{c}\n")

    def to_text(self, path: str):
        with open(path, "w") as f:
            for p, nd, hr, c in self.periods():
                f.write(f"{p}\t{nd}\t{hr}\t{c}\n")


def recall_precision_at_k(recommended: Dict[int, Sequence[int]], relevant: Dict[int, set], k: int = 5):
    rec_sum = prec_sum = 0.0
    n = 0
    for u, rel in relevant.items():
        if not rel or u not in recommended:
            continue
        top = list(recommended[u])[:k]
        hit = len(set(top) & rel)
        rec_sum += hit / len(rel)
        prec_sum += hit / k
        n += 1
    return (rec_sum / max(n, 1), prec_sum / max(n, 1))


def top_k_from_factors(users: Dict[int, np.ndarray], items: Dict[int, np.ndarray], k: int = 5,
                       exclude: Optional[Dict[int, set]] = None) -> Dict[int, List[int]]:
    """Brute-force top-K per user from dumped factors (the notebooks' recommendation step)."""
    ids = np.array(sorted(items))
    M = np.stack([items[i] for i in ids]) if len(ids) else np.zeros((0, 1))
    out = {}
    for u, vec in users.items():
        s = M @ vec
        order = np.argsort(-s, kind="stable")
        ex = exclude.get(u, set()) if exclude else set()
        out[u] = [int(ids[j]) for j in order if int(ids[j]) not in ex][:k]
    return out


# ------------------------------------------------------------------ runtime metrics
class Counters:
    def __init__(self):
        self.c = defaultdict(float)

    def add(self, name: str, v: float = 1.0):
        self.c[name] += v

    def snapshot(self) -> Dict[str, float]:
        return dict(self.c)


class StageTimer:
    """Per-stage timing; ``device=True`` uses HIP events recorded on the stream
    current at the stage (no host sync per stage; a stage opened under
    ``torch.cuda.stream(side)`` is timed on ``side``).  ``step_end()`` closes
    a step so ``per_step_ms()`` can report every stage of every step."""

    def __init__(self, device: bool = False):
        self.device = device
        self.wall = defaultdict(float)
        self.events: Dict[str, list] = defaultdict(list)
        self._step: Dict[str, list] = defaultdict(list)
        self._steps: list = []

    @contextmanager
    def stage(self, name: str):
        if self.device:
            import torch

            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            try:
                yield
            finally:
                b.record()
                self.events[name].append((a, b))
                self._step[name].append((a, b))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                dt = time.perf_counter() - t0
                self.wall[name] += dt
                self._step[name].append(dt)

    def step_end(self):
        self._steps.append(self._step)
        self._step = defaultdict(list)

    @staticmethod
    def _ms(x) -> float:
        if isinstance(x, tuple):
            return x[0].elapsed_time(x[1])
        return x * 1e3

    def per_step_ms(self) -> list:
        """``[{stage: ms}]`` per closed step (syncs the device once)."""
        if self.device:
            import torch

            torch.cuda.synchronize()
        return [{k: sum(self._ms(x) for x in v) for k, v in st.items()} for st in self._steps]

    def totals_ms(self) -> Dict[str, float]:
        out = {k: v * 1e3 for k, v in self.wall.items()}
        if self.events:
            import torch

            torch.cuda.synchronize()
            for k, evs in self.events.items():
                out[k] = out.get(k, 0.0) + sum(a.elapsed_time(b) for a, b in evs)
        return out


class JsonlWriter:
    def __init__(self, path: str):
        self.f = open(path, "a")

    def write(self, **record):
        record.setdefault("time", time.time())
        self.f.write(json.dumps(record) + "\n")
        self.f.flush()

    def close(self):
        self.f.close()
