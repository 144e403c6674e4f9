#!/usr/bin/env python3
"""The headline step's two halves timed apart and together (one MI355X).

    python bench/probe_partition.py [--steps 20] [--warmup 3]

On the bench.py model (10M x 1M, rank 64, 64M ratings per step, N = 1, local
exchange, tiled SGD with the partition of batch k+1 on a side stream beside the SGD
of batch k) this prints one JSON line with

* ``partition_ms``: ``TilePartitioner.run`` alone (count, scans, level-1 and level-2
  scatters), back to back on the compute stream;
* ``sgd_ms``: the tiled SGD of one staged batch alone (``user_phases`` pair launches);
* ``step_ms``: ``DistributedMF.step`` as bench.py times it (both overlapped);
* ``overlap_saving_ms`` = partition + sgd - step.

The kernel variants of ``csrc/kernels/mf_tiled.hip`` are A/B'd by pointing
``FPS_KERNELS_SO`` at a variant build (``csrc/build.py --variant``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=64 << 20)
    ap.add_argument("--only", default="part,sgd,step", help="comma list of part / sgd / step")
    ap.add_argument("--user-phases", type=int, default=0, help="0: MFConfig's choice")
    a = ap.parse_args(argv)

    import torch

    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings

    dev = torch.device("cuda", 0)
    cfg = MFConfig(num_users=a.users, num_items=a.items, dim=64, learning_rate=0.01, user_phases=a.user_phases)
    model = DistributedMF(cfg)
    assert model.sgd_mode == "tiled" and model.exchange == "local", (model.sgd_mode, model.exchange)
    data = SyntheticRatings(a.users, a.items, a.batch * 2, 0, 1, device=dev)
    only = set(a.only.split(","))
    out = {"users": a.users, "items": a.items, "batch": a.batch, "user_phases": model.user_phases,
           "tile_R": model.tile_R, "tile_T": model.tile_T, "kernels_so": os.environ.get("FPS_KERNELS_SO")}

    def timed(fn, n):
        for i in range(a.warmup):
            fn(i)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            fn(a.warmup + i)
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / n

    tiler = model._tilers[0]
    if "part" in only:
        out["partition_ms"] = timed(lambda i: tiler.run(*data.batch(i, a.batch)), a.steps)
    if "sgd" in only:
        ptr, rec = tiler.run(*data.batch(0, a.batch))
        out["sgd_ms"] = timed(lambda i: model._tiled_sgd((ptr, rec, None)), a.steps)
    if "step" in only:
        def st(i):
            model.step(*data.batch(i, a.batch))

        for i in range(a.warmup):
            st(i)
        model.flush()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.steps):
            st(a.warmup + i)
        model.flush()
        e1.record()
        torch.cuda.synchronize(dev)
        out["step_ms"] = e0.elapsed_time(e1) / a.steps
        out["updates_per_s"] = a.batch / out["step_ms"] * 1e3
    if {"partition_ms", "sgd_ms", "step_ms"} <= out.keys():
        out["overlap_saving_ms"] = out["partition_ms"] + out["sgd_ms"] - out["step_ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
