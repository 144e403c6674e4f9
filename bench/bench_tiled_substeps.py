#!/usr/bin/env python3
"""Per-GPU compute of one MF step at the shapes of an N-GPU rotation run, on one GPU.

At N GPUs every rank holds 10M/N users, takes 64M ratings per step and runs
2N sub-steps of ``mf_sgd_tiled`` over item blocks of 1M/(2N) rows
(``parallel/rotation.py``).  This times exactly those launches (no transport)
so the per-GPU compute efficiency of the scaling run can be read on one GPU:

    python bench/bench_tiled_substeps.py [--ws 1,2,4,8] [--batch 67108864]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", default="1,2,4,8")
    ap.add_argument("--batch", type=int, default=1 << 26)
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()

    import torch

    from flink_parameter_server_1_amd import ops
    from flink_parameter_server_1_amd.parallel.rotation import block_rows, shard_halves

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    for W in [int(x) for x in a.ws.split(",")]:
        n_users = -(-a.users // W)
        U = torch.empty((n_users, a.dim), device=dev).uniform_(-0.01, 0.01, generator=g)
        rows = block_rows(a.items, W)
        bmax = max(rows)
        R = ops.tile_rows_for(a.dim, bmax, W)
        T = -(-bmax // R)
        blocks = [torch.empty((r, a.dim), device=dev).uniform_(-0.01, 0.01, generator=g) for r in rows]
        uid = torch.randint(0, n_users, (a.batch,), device=dev, dtype=torch.int32, generator=g)
        iid = torch.randint(0, a.items, (a.batch,), device=dev, dtype=torch.int32, generator=g)
        rt = torch.rand(a.batch, device=dev, generator=g)
        tiler = ops.TilePartitioner(W, shard_halves(a.items, W), R, T, dev, rec8=n_users < (1 << 24))
        ptr, rec = tiler.run(uid, iid, rt)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        best_sgd = best_part = 1e30
        for _ in range(a.reps):
            ev[0].record()
            ptr, rec = tiler.run(uid, iid, rt)
            ev[1].record()
            for b in range(2 * W):
                ops.mf_sgd_tiled(U, blocks[b], rec, ptr, b, T, R, 0.01, 0.0)
            ev[2].record()
            torch.cuda.synchronize()
            best_part = min(best_part, ev[0].elapsed_time(ev[1]))
            best_sgd = min(best_sgd, ev[1].elapsed_time(ev[2]))
        print(json.dumps({"W": W, "R": R, "T": T, "workgroups_per_substep": T, "substeps": 2 * W,
                          "partition_ms": round(best_part, 3), "sgd_ms": round(best_sgd, 3),
                          "sgd_updates_per_s": a.batch / best_sgd * 1e3}), flush=True)
        del U, blocks, uid, iid, rt, tiler, ptr, rec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
