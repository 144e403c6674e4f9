#!/usr/bin/env python3
"""Drive single kernels at production sizes for counter passes (``rocprofv3 --pmc``).

    python bench/probe_kernels.py {hash,route,coord} [--reps 5]

* ``hash``  -- the device hash-table shard (``parallel/hash_table.py``,
  ``csrc/kernels/hash_table.hip``): 4M sparse int32 ids per call, looked up with
  first-touch insert into a shard of 16M slots (~25 % new ids per call after the
  first), dim 32 (``rows_for`` = lookup-or-insert + row init);
* ``route`` -- the request-plan routing kernel (``ops.DedupWorkspace.route``): 4M
  keys over a 1B id space to 8 owners (the PA PS path at W = 8);
* ``coord`` -- the bf16 LEMP scorer with the COORD bound evaluated
  (``ops.score_filter_bf16`` via ``LempTopK``): 1M axis-dominated items of dim 64,
  4096 queries over 8 focus coordinates (the bound skips block pairs here).

Each mode runs ``--reps`` calls after one warm-up call and prints one JSON line
with the mean wall time per call.
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
    ap.add_argument("mode", choices=["hash", "route", "coord"])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args(argv)

    import torch

    from flink_parameter_server_1_amd import ops

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    info = {}
    if a.mode == "hash":
        from flink_parameter_server_1_amd.parallel.hash_table import HashShardTable

        t = HashShardTable(32, device=dev, capacity=8_000_000, init=("uniform", -0.01, 0.01))
        n = 4 << 20
        pool = torch.randint(-(1 << 31), (1 << 31) - 1, (12 << 20,), generator=g, device=dev, dtype=torch.int64)
        pool = pool.to(torch.int32)

        def call(i):
            s = (i * 3 * n // 4) % (pool.numel() - n)  # a quarter of each call's ids are new
            t.rows_for(pool[s:s + n])
        info["table_rows"] = lambda: int(t.count.item())
    elif a.mode == "route":
        F, W, n = 1_000_000_000, 8, 4 << 20
        ws = ops.DedupWorkspace(F, W, 1, -(-F // W), dev)
        keys = (torch.rand(n, generator=g, device=dev) ** 2 * F).to(torch.int32)

        def call(i):
            ws.route(keys)
    else:
        from flink_parameter_server_1_amd.models.mf.pruning import LEMPPruningStrategy
        from flink_parameter_server_1_amd.models.mf.topk_fast import LempTopK

        N, D, B, k = 1_000_000, 64, 4096, 100
        axis = torch.randint(0, D, (N,), generator=g, device=dev)
        X = torch.randn(N, D, generator=g, device=dev) * 0.05
        X[torch.arange(N, device=dev), axis] += 1.0
        X *= torch.rand(N, 1, generator=g, device=dev) ** 2 + 0.05
        qa = torch.randint(0, 8, (B,), generator=g, device=dev)
        Q = torch.randn(B, D, generator=g, device=dev) * 0.05
        Q[torch.arange(B, device=dev), qa] += 1.0
        idx = LempTopK(torch.arange(N, device=dev), X, 65536, strategy=LEMPPruningStrategy.from_string("coord"))

        def call(i):
            idx.query(Q, k)
        info["coord_block_pairs_scored_skipped"] = lambda: idx.coord_stats.tolist()
    call(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.reps):
        call(i + 1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    out = {"probe": a.mode, "reps": a.reps, "ms_per_call": dt * 1e3}
    out.update({k: v() for k, v in info.items()})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
