#!/usr/bin/env python3
"""The N-GPU headline step in the virtual world: N rank threads on ONE GPU over the
RCCL-semantics transport (``parallel/vworld.py``) with modelled xGMI transfer times.

    python bench/bench_vworld.py --world 8 [--batch 67108864] [--steps 6] [--link-gbps 50]
                                 [--dilate N] [--exchange rotate|ps]

Each rank runs the real ``DistributedMF`` step of ``bench.py`` (tile-partitioned SGD,
bidirectional item-block rotation) on its own compute stream; every block transfer
runs on a link stream behind a device sleep of ``latency + bytes / link_gbps``.  The
ranks share the GPU, so each rank's compute runs ~N x slower than on its own GPU;
``--dilate`` (default N) stretches the modelled transfers by the same factor so the
compute / transfer ratio is the real job's.  Reported per rank: the wall time per
step (all ranks together) and ``comm_wait_ms_per_step`` -- the time the rank's compute
stream waited on transfers (HIP events around each wait, ``RingRotation.wait_ms``);
``exposed`` = wait / step.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--batch", type=int, default=1 << 26, help="ratings per rank per step")
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--link-gbps", type=float, default=50.0, help="modelled GB/s of one link direction")
    ap.add_argument("--latency-us", type=float, default=10.0)
    ap.add_argument("--dilate", type=float, default=None, help="transfer-time stretch (default: world)")
    ap.add_argument("--exchange", default="rotate", choices=["rotate", "ps"])
    ap.add_argument("--rotation", default="bidir", choices=["bidir", "ring"])
    ap.add_argument("--mode", default="async", choices=["async", "sync"])
    ap.add_argument("--no-delay", action="store_true",
                    help="control run: transfers as soon as both sides posted (what remains is rank skew)")
    ap.add_argument("--traceback-s", type=float, default=0.0,
                    help="dump every thread's Python stack to stderr every this many seconds (hang diagnosis)")
    a = ap.parse_args(argv)
    if a.traceback_s > 0:
        import faulthandler

        faulthandler.dump_traceback_later(a.traceback_s, repeat=True, file=sys.stderr)

    import torch

    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.vworld import run_virtual

    dilate = float(a.world) if a.dilate is None else a.dilate
    cuda = torch.cuda.is_available()

    def sync(all_streams=False):
        if cuda:
            torch.cuda.synchronize() if all_streams else torch.cuda.current_stream().synchronize()
    barrier = __import__("threading").Barrier(a.world)

    def rank_main(comm):
        cfg = MFConfig(num_users=a.users, num_items=a.items, dim=a.dim, exchange=a.exchange, rotation=a.rotation)
        m = DistributedMF(cfg, comm)
        data = SyntheticRatings(a.users, a.items, a.batch, comm.rank, comm.world, device=comm.device)
        batch = data.batch(0, a.batch)
        for _ in range(a.warmup):
            m.step(*batch)
        m.flush()
        if m.exchange == "rotate":
            m.rot.wait_ms()
        sync(True)
        barrier.wait()
        t0 = time.perf_counter()
        for k in range(a.steps):
            m.step(*batch)
            if comm.rank == 0:
                print(f"[vworld] rank 0 enqueued step {k}", file=sys.stderr, flush=True)
        m.flush()
        sync()
        barrier.wait()
        sync(True)
        dt = time.perf_counter() - t0
        wait = m.rot.wait_ms() / a.steps if m.exchange == "rotate" else 0.0
        return {"ms_per_step": dt / a.steps * 1e3, "comm_wait_ms_per_step": wait,
                "rotation_bytes_sent": m.rot.bytes_sent if m.exchange == "rotate" else None,
                "a2a_bytes_sent": comm.bytes_sent, "sgd_mode": m.sgd_mode}

    res, vw = run_virtual(rank_main, a.world, mode=a.mode, link_gbps=a.link_gbps, latency_us=a.latency_us,
                          dilate=dilate, return_world=True, timeout_s=1000, delay=not a.no_delay)
    step = max(r["ms_per_step"] for r in res)
    waits = [r["comm_wait_ms_per_step"] for r in res]
    link_ms = sum(vw.link_us.values()) / 1e3 / max(len(vw.link_us), 1) / (a.steps + a.warmup)
    out = {
        "bench": "vworld", "world": a.world, "exchange": a.exchange, "rotation": a.rotation, "mode": a.mode,
        "batch_per_rank": a.batch, "users": a.users, "items": a.items, "dim": a.dim, "steps": a.steps,
        "link_gbps": a.link_gbps, "latency_us": a.latency_us, "dilate": dilate, "delay": not a.no_delay,
        "ms_per_step_all_ranks_one_gpu": step,
        "comm_wait_ms_per_step_per_rank": waits,
        "exposed_wait_fraction_max": max(waits) / step if step else None,
        "modelled_transfer_ms_per_step_per_link": link_ms,
        "transfers": vw.transfers, "sgd_mode": res[0]["sgd_mode"],
        "rotation_bytes_sent_rank0": res[0]["rotation_bytes_sent"],
        "note": "N ranks share one GPU: per-rank compute ~N x the real per-GPU step; transfers dilated x dilate",
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
