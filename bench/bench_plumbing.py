#!/usr/bin/env python3
"""BASELINE config #1: 1k x 1k rank-8 MF-SGD, 1 worker + 1 PS, CPU plumbing (no GPU).

    python bench/bench_plumbing.py [--ratings 100000] [--engine record|tensor|both]

* ``record``: the per-record engine (``LocalRuntime``) running ``ps_online_mf``
  exactly like the reference job (``M/matrix/factorization/PSOnlineMatrixFactorization.scala``),
  one worker + one PS subtask, every rating a pull + a push through the
  mailboxes -- measures the protocol overhead per record.
* ``native``: the same per-record job (same messages, schedule and semantics,
  tested equal to ``record`` on the folded model) in the C++ record engine
  (``csrc/host/record_engine.cpp``, ``models.mf.native.ps_online_mf_native``).
* ``tensor``: the same model on the tensor engine on CPU (``DistributedMF`` with
  the PyTorch reference ops), micro-batches of ``--batch`` ratings.

Reports rating updates/s for each engine and the final training RMSE
(synthetic ratings from a hidden rank-8 model, so RMSE must fall).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _ratings(n, users, items, rank, seed):
    import numpy as np

    from flink_parameter_server_1_amd.models.mf.core import Rating

    rng = np.random.default_rng(seed)
    U = rng.random((users, rank)) / rank ** 0.5
    V = rng.random((items, rank)) / rank ** 0.5
    u = rng.integers(0, users, n)
    i = rng.integers(0, items, n)
    r = (U[u] * V[i]).sum(1)
    return [Rating(int(a), int(b), float(c), t) for t, (a, b, c) in enumerate(zip(u, i, r))], (u, i, r)


def run_record(n, users, items, rank, lr):
    import numpy as np

    from flink_parameter_server_1_amd.core.messages import Left, Right
    from flink_parameter_server_1_amd.models.mf.apps import ps_online_mf

    data, (u, i, r) = _ratings(n, users, items, rank, 1)
    t0 = time.perf_counter()
    out = ps_online_mf(data, num_factors=rank, range_min=0.0, range_max=0.3, learning_rate=lr,
                       worker_parallelism=1, ps_parallelism=1, pull_limit=1600, seed=7)
    dt = time.perf_counter() - t0
    U, V = {}, {}
    for e in out:  # last-writer-wins fold of the output stream (C51)
        if isinstance(e, Left):
            U[e.value[0]] = np.asarray(e.value[1])
        elif isinstance(e, Right):
            V[e.value[0]] = np.asarray(e.value[1])
    err = [r[k] - float(np.dot(U[u[k]], V[i[k]])) for k in range(n) if u[k] in U and i[k] in V]
    return {"engine": "record", "updates_per_s": n / dt, "seconds": dt,
            "rmse": float(np.sqrt(np.mean(np.square(err)))) if err else None}


def run_native(n, users, items, rank, lr, reps=5):
    import numpy as np

    from flink_parameter_server_1_amd.models.mf.native import ps_online_mf_native

    _, (u, i, r) = _ratings(n, users, items, rank, 1)
    best = None
    for _ in range(reps):  # best of a few runs (sub-second job)
        t0 = time.perf_counter()
        res = ps_online_mf_native(u, i, r, num_factors=rank, range_min=0.0, range_max=0.3, learning_rate=lr,
                                  worker_parallelism=1, ps_parallelism=1, pull_limit=1600, seed=7)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    U, V = res.users(), res.items()
    err = [r[k] - float(np.dot(U[u[k]], V[i[k]])) for k in range(n)]
    return {"engine": "native-record", "updates_per_s": n / best, "seconds": best,
            "rmse": float(np.sqrt(np.mean(np.square(err)))), "messages": res.stats}


def run_tensor(n, users, items, rank, lr, batch):
    import torch

    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig

    _, (u, i, r) = _ratings(n, users, items, rank, 1)
    uid = torch.as_tensor(u, dtype=torch.int32)
    iid = torch.as_tensor(i, dtype=torch.int32)
    rat = torch.as_tensor(r, dtype=torch.float32)
    m = DistributedMF(MFConfig(num_users=users, num_items=items, dim=rank, learning_rate=lr, range_min=0.0,
                               range_max=0.3))
    before = m.rmse(uid, iid, rat)
    t0 = time.perf_counter()
    for s in range(0, n, batch):
        m.step(uid[s:s + batch], iid[s:s + batch], rat[s:s + batch])
    m.flush()
    dt = time.perf_counter() - t0
    return {"engine": "tensor-cpu", "updates_per_s": n / dt, "seconds": dt, "rmse_before": before,
            "rmse": m.rmse(uid, iid, rat)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ratings", type=int, default=100_000)
    ap.add_argument("--users", type=int, default=1000)
    ap.add_argument("--items", type=int, default=1000)
    ap.add_argument("--rank", type=int, default=8)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--batch", type=int, default=1000)
    ap.add_argument("--engine", default="all", choices=["record", "native", "tensor", "all"])
    a = ap.parse_args(argv)
    res = []
    if a.engine in ("record", "all"):
        res.append(run_record(a.ratings, a.users, a.items, a.rank, a.lr))
    if a.engine in ("native", "all"):
        res.append(run_native(a.ratings, a.users, a.items, a.rank, a.lr))
    if a.engine in ("tensor", "all"):
        res.append(run_tensor(a.ratings, a.users, a.items, a.rank, a.lr, a.batch))
    for x in res:
        print(json.dumps({"metric": "MF-SGD rating updates/sec, 1k x 1k rank-8, 1 worker + 1 PS (CPU plumbing)",
                          "value": x["updates_per_s"], "unit": "updates/s", "n_gpus": 0, "higher_is_better": True,
                          "dtype": "fp32" if x["engine"] == "tensor-cpu" else "fp64", "data": "synthetic rank-8 ratings",
                          **x}), flush=True)


if __name__ == "__main__":
    main()
