#!/usr/bin/env python3
"""Online MF + top-K serving (psOnlineLearnerAndGenerator) on the tensor engine.

    python bench/bench_mf_topk.py [--users 1000000] [--items 1000000] [--dim 64] [--batch 4096]
    (N > 1 under torch.distributed.run: items sharded over the ranks, queries broadcast)

Every broadcast rating is a top-K query (MFMA LEMP scoring over the local item
shard, all_gather + merge with the user's seen items removed) and a learning
update on the rank owning the item (SGD on the local item, user delta pushed to
the PS: add_renorm).  Reports top-K queries/s and learning updates/s for the
whole job; synthetic ratings, random-init factors, the item catalogue warm.
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
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4096, help="broadcast ratings (queries) per micro-batch")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--worker-k", type=int, default=75)
    ap.add_argument("--negatives", type=int, default=2)
    ap.add_argument("--memory", type=int, default=16)
    ap.add_argument("--bucket", type=int, default=65536)
    ap.add_argument("--seed-items", type=int, default=None, help="LempTopK.seed_items (unfused first segment)")
    ap.add_argument("--max-segment", type=int, default=None, help="LempTopK.max_segment (largest fused segment)")
    ap.add_argument("--unfused", action="store_true",
                    help="torch chains for the merge / SGD and eager scans (the A/B reference)")
    ap.add_argument("--capacity", action="store_true",
                    help="fixed-shape PS plans (capacity = the batch): at N > 1 no count exchange read on the host")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args(argv)

    import torch

    from flink_parameter_server_1_amd.core.tensor_engine import TensorRuntime
    from flink_parameter_server_1_amd.models.mf.topk_tensor import OnlineMFTopKWorker
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogic

    from flink_parameter_server_1_amd.models.mf.topk_fast import LempTopK

    if a.seed_items:
        LempTopK.seed_items = a.seed_items
    if a.max_segment:
        LempTopK.max_segment = a.max_segment
    comm = Comm.init_from_env()
    dev = comm.device
    worker = OnlineMFTopKWorker(a.items, a.dim, 0.01, K=a.k, worker_k=a.worker_k, memory=a.memory,
                                negative_sample_rate=a.negatives, bucket_size=a.bucket, range_min=-0.1,
                                range_max=0.1, prefill_items=True, num_users=a.users)
    if a.unfused:
        worker.fused = False
        os.environ["FPS_TOPK_GRAPH"] = "0"
    logic = DeviceSimplePSLogic(a.users, a.dim, op="add_renorm", init=("uniform", -0.1, 0.1))
    logic.emit = "none"  # the benchmark keeps no output stream of the user updates
    rt = TensorRuntime(comm, staleness=0, output_sink=lambda e: None,
                       capacity=a.batch if a.capacity else None).start(worker, logic)
    g = torch.Generator(device=dev)
    g.manual_seed(5)  # the same broadcast batches on every rank

    def batch(s):
        return (torch.randint(0, a.users, (a.batch,), generator=g, device=dev),
                torch.randint(0, a.items, (a.batch,), generator=g, device=dev),
                torch.arange(s * a.batch, (s + 1) * a.batch, device=dev),
                torch.rand(a.batch, generator=g, device=dev))

    data = [batch(s) for s in range(4)]

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for s in range(a.warmup):
        rt.submit(data[s % 4])
    comm.barrier()
    sync()
    served0, trained0 = worker.served, worker.trained  # (synchronised above: read before the clock starts)
    t0 = time.perf_counter()
    for s in range(a.steps):
        rt.submit(data[s % 4])
    sync()
    comm.barrier()
    dt = comm.max_over_ranks(time.perf_counter() - t0)
    queries = (worker.served - served0)  # the same broadcast queries on every rank
    learned = comm.sum_over_ranks(float(worker.trained - trained0))
    if comm.rank == 0:
        print(json.dumps({
            "metric": "online MF + top-K: top-K queries/sec (whole node)", "value": queries / dt,
            "unit": "queries/s", "learning_updates_per_s": learned / dt, "n_gpus": comm.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "strong",
            "dtype": "fp32", "scorer": _scorer(), "data": "synthetic ratings, random-init factors (warm item catalogue)",
            "config": {"users": a.users, "items": a.items, "dim": a.dim, "k": a.k, "worker_k": a.worker_k,
                       "batch": a.batch, "negatives": a.negatives, "memory": a.memory, "bucket": a.bucket,
                       "seed_items": LempTopK.seed_items, "max_segment": LempTopK.max_segment,
                       "fused": not a.unfused, "fixed_plans": bool(a.capacity) and comm.world > 1},
        }), flush=True)
    comm.shutdown()  # every rank leaves the process group together


if __name__ == "__main__":
    main()
