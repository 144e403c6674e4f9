#!/usr/bin/env python3
"""Top-K recommendation throughput (psTopKGenerator on the GPU): LEMP bucket scan + MFMA scoring.

    python bench/bench_topk.py [--items 1000000] [--dim 64] [--queries 4096] [--k 100]
    (N > 1 under torch.distributed.run: items sharded over the ranks, partial top-Ks merged)

Item vectors are random with a long-tailed length distribution (real MF factors
have it: popular items get long vectors), so the LEMP length bound prunes
buckets.  Reports queries/s for the whole job, the fraction of buckets
scanned, and checks a sample of queries against brute force.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _scorer() -> str:
    """Which top-K scan ran: the default bf16 MFMA filter + exact fp32 re-score
    (results bit-identical to the fp32 scan) or the fp32 scorer (FPS_TOPK_BF16=0)."""
    if os.environ.get("FPS_TOPK_BF16", "1") == "0":
        return "fp32 MFMA scan"
    return "bf16 MFMA filter (proven margin) + fp32 MFMA re-score: exact"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--queries", type=int, default=4096, help="query users per batch per GPU")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--bucket", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--strategy", default="length",
                    help="LEMP pruning applied per 32-item block on the device: length | coord | lc:T | li:N:T | "
                         "incr:N (LEMPPruningStrategy.fromString syntax; li / incr run the length bound)")
    ap.add_argument("--sync", action="store_true",
                    help="read every batch's overflow flag before the next batch is enqueued (the round-4 loop); "
                         "default: query_async, batch k's result taken after batch k + 1 is enqueued")
    a = ap.parse_args(argv)

    import torch

    from flink_parameter_server_1_amd.models.mf.topk_fast import DistributedTopK
    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm.init_from_env()
    dev = comm.device
    g = torch.Generator(device=dev)
    g.manual_seed(17 + comm.rank)
    n_local = (a.items - comm.rank + comm.world - 1) // comm.world
    ids = comm.rank + comm.world * torch.arange(n_local, device=dev)
    scale = torch.rand(n_local, 1, generator=g, device=dev) ** 4  # long-tailed vector lengths
    vecs = torch.randn(n_local, a.dim, generator=g, device=dev) * scale
    from flink_parameter_server_1_amd.models.mf.pruning import LEMPPruningStrategy

    strategy = LEMPPruningStrategy.from_string(a.strategy)
    topk = DistributedTopK(ids, vecs, comm, bucket_size=a.bucket, strategy=strategy)
    gq = torch.Generator(device=dev)
    gq.manual_seed(5)  # same query batch on every rank (broadcast users)
    queries = [torch.randn(a.queries, a.dim, generator=gq, device=dev) for _ in range(4)]

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def run(n):
        if a.sync:
            for s in range(n):
                topk.query(queries[s % 4], a.k)
            return
        prev = None
        for s in range(n):  # enqueue batch s, then complete batch s - 1: the host never drains the device
            f = topk.query_async(queries[s % 4], a.k)
            if prev is not None:
                prev.result()
            prev = f
        if prev is not None:
            prev.result()

    run(a.warmup)
    comm.barrier()
    sync()
    scanned0 = topk.local.buckets_scanned
    t0 = time.perf_counter()
    run(a.steps)
    sync()
    comm.barrier()
    dt = comm.max_over_ranks(time.perf_counter() - t0)
    n_buckets = -(-n_local // a.bucket)
    scanned = (topk.local.buckets_scanned - scanned0) / max(a.steps, 1)
    # exactness spot check on this rank's shard (brute force)
    from flink_parameter_server_1_amd.models.mf.topk_fast import LempTopK

    q = queries[0][:64]
    s_l, i_l = LempTopK(ids, vecs, a.bucket).query(q, a.k)
    ref = torch.topk(q @ vecs.T, a.k, dim=1)
    exact = bool(torch.allclose(s_l, ref.values, rtol=1e-4, atol=1e-4))
    if comm.rank == 0:
        print(json.dumps({
            "metric": "top-K recommendation queries/sec (whole node)", "value": a.queries * a.steps / dt,
            "unit": "queries/s", "n_gpus": comm.world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "pipelined_results": not a.sync, "scaling": "strong", "dtype": "fp32", "scorer": _scorer(),
            "data": "synthetic long-tailed item factors, random queries",
            "buckets_scanned_per_query_batch": scanned, "buckets_per_shard": n_buckets, "exact_vs_brute_force": exact,
            "coord_block_pairs_scored_skipped": topk.local.coord_stats.tolist()
            if topk.local.coord_stats is not None else None,
            "config": {"items": a.items, "dim": a.dim, "k": a.k, "query_batch": a.queries, "bucket": a.bucket,
                       "strategy": a.strategy},
        }), flush=True)
    comm.shutdown()  # every rank leaves the process group together


if __name__ == "__main__":
    main()
