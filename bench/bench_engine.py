#!/usr/bin/env python3
"""Tensor-engine plumbing on the GPU: the public batched API with a trivial user worker.

    python bench/bench_engine.py [--keys 10000000] [--dim 64] [--batches 1,64,4096,262144]
    (N > 1 under torch.distributed.run: keys hash-sharded over the ranks, all-to-all exchange)

A ``FunctionBatchedWorkerLogic`` pulls the keys of every micro-batch and pushes
a constant delta per pulled row (``DeviceSimplePSLogic(op="add")``), so the
numbers measure the engine itself -- dedup, count exchange, key / row / delta
all-to-alls, gather, apply, the host control loop -- as micro-batches/s and
pulled+pushed keys/s per micro-batch size (the config #1 plumbing question on
the device path).  Synthetic uniform keys.

``--capacity`` switches to fixed-shape plans (``TensorPS.capacity`` = the batch
size): at world > 1 no split size reaches the host and ``--graph`` captures the
steps with their RCCL all-to-alls.  ``--loopback`` (world 1) runs those
all-to-alls through a one-rank RCCL group, so a one-GPU box measures the captured
world > 1 step shape with real RCCL kernels in it.
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
    ap.add_argument("--keys", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--batches", default="1,64,4096,262144")
    ap.add_argument("--seconds", type=float, default=2.0, help="timed seconds per micro-batch size")
    ap.add_argument("--staleness", type=int, default=0)
    ap.add_argument("--graph", action="store_true", help="replay captured hipGraph steps (core.step_graph)")
    ap.add_argument("--capacity", action="store_true", help="fixed-shape plans, capacity = the batch size")
    ap.add_argument("--loopback", action="store_true",
                    help="world 1: all-to-alls through a one-rank RCCL group (implies --capacity)")
    a = ap.parse_args(argv)

    import torch

    from flink_parameter_server_1_amd.api.batched import FunctionBatchedWorkerLogic
    from flink_parameter_server_1_amd.core.tensor_engine import TensorRuntime
    from flink_parameter_server_1_amd.parallel.comm import Comm
    from flink_parameter_server_1_amd.ps.device_logics import DeviceSimplePSLogic

    comm = Comm.init_from_env()
    dev = comm.device
    if a.loopback:
        import socket

        import torch.distributed as dist

        if comm.world != 1 or dev.type != "cuda":
            raise SystemExit("--loopback is a one-GPU, world-1 mode")
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
        comm = Comm(device=dev)
        comm.loopback = True
        a.capacity = True

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    results = []
    for B in [int(x) for x in a.batches.split(",")]:
        worker = FunctionBatchedWorkerLogic(lambda keys, ps: ps.pull(keys),
                                            lambda pulled, ps: ps.push_unique(torch.full(
                                                (pulled.n_unique, a.dim), 1e-3, device=pulled.rows.device)),
                                            graph_safe=True)
        logic = DeviceSimplePSLogic(a.keys, a.dim, op="add", init=("zeros",))
        logic.emit = "none"
        rt = TensorRuntime(comm, staleness=a.staleness, output_sink=lambda e: None,
                           graph=a.graph, capacity=B if a.capacity else None).start(worker, logic)
        g = torch.Generator(device=dev)
        g.manual_seed(11 + comm.rank)
        pool = [torch.randint(0, a.keys, (B,), generator=g, device=dev) for _ in range(8)]
        for s in range(5):
            rt.submit(pool[s % 8])
        rt.pipe.drain() if hasattr(rt, "pipe") and hasattr(rt.pipe, "drain") else None
        sync()
        comm.barrier()
        # a fixed step count per size (the same on every rank), from a rough calibration
        t0 = time.perf_counter()
        for s in range(20):
            rt.submit(pool[s % 8])
        sync()
        per = max((time.perf_counter() - t0) / 20, 1e-6)
        steps = int(comm.max_over_ranks(min(100000.0, max(20.0, a.seconds / per))))
        comm.barrier()
        sync()
        t0 = time.perf_counter()
        for s in range(steps):
            rt.submit(pool[s % 8])
        if hasattr(rt, "pipe") and hasattr(rt.pipe, "drain"):
            rt.pipe.drain()
        sync()
        comm.barrier()
        dt = comm.max_over_ranks(time.perf_counter() - t0)
        results.append({"batch": B, "steps": steps, "graph_replays": rt.graphs.replays if rt.graphs else 0, "micro_batches_per_s": steps / dt,
                        "keys_per_s": comm.world * steps * B / dt, "us_per_step": dt / steps * 1e6})
        if rt.graphs is not None:
            rt.graphs.release()
        del rt
    if a.loopback:  # the graphs that reference the communicator are gone: tear it down
        import gc

        import torch.distributed as dist

        gc.collect()
        sync()
        dist.destroy_process_group()
    if comm.rank == 0:
        print(json.dumps({"metric": "tensor-engine plumbing: micro-batches/s and keys/s (whole node)",
                          "n_gpus": comm.world, "dtype": "fp32", "data": "synthetic uniform keys",
                          "config": {"keys": a.keys, "dim": a.dim, "staleness": a.staleness, "graph": a.graph,
                                     "fixed_plans": bool(a.capacity), "rccl_loopback": a.loopback}, "results": results}),
              flush=True)


if __name__ == "__main__":
    main()
