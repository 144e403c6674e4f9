#!/usr/bin/env python3
"""Per-GPU step of an N-GPU rotation run, measured on ONE GPU.

At N GPUs every rank holds 10M/N users, takes ``--batch`` ratings per step
(weak scaling) and runs 2N sub-steps of the tiled SGD over the item blocks it
holds (``parallel/rotation.py``: two counter-rotating rings of 1M/(4N)-row
blocks by default).  ``MFConfig(emulate_world=N)`` runs rank 0's exact schedule
with every block resident (``EmulatedRotation``): the same partition and the
same launches per sub-step as one GPU of the real job, without the transfers.
Comparing the emulated step with the N = 1 step separates "compute slower at
N" from "transfer exposed" before an N-GPU node runs the real thing.  With
``--link-gbps`` the transfers are modelled too (``rotation._SymmetricLinks``:
rank-symmetric timing, a device-timed link delay and a real device copy per block)
and ``comm_wait_ms_per_step`` is the time the compute stream waited for them.

    python bench/bench_emulate_world.py [--ws 1,2,4,8] [--steps 20 --warmup 5]

One JSON line per N: ms_per_step, per-GPU updates/s, ratio to N = 1.

Each N runs in a fresh child interpreter: a process that has already built models of
other world sizes holds more HIP streams than the 4 hardware queues a process gets, and
the queue an N-rank model's streams then share with each other is luck -- the same N = 8
emulation measured 7.1 ms alone and 9.2 ms after N = 2 and 4 in one process
(``profiles/r6_link_model.md``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", default="1,2,4,8")
    ap.add_argument("--batch", type=int, default=1 << 26)
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pool", type=int, default=4)
    ap.add_argument("--rotation", default="bidir", choices=["bidir", "ring"])
    ap.add_argument("--link-gbps", type=float, default=0.0,
                    help="model each sub-step's transfers on links of this rate (EmulatedRotation: rank-symmetric "
                         "timing, a one-wave device sleep for the link time + a real device copy); 0 = no transfers")
    ap.add_argument("--latency-us", type=float, default=5.0)
    ap.add_argument("--user-update", default="auto", choices=["auto", "store", "sc1", "atomic"],
                    help="auto = what bench.py runs at every world size (store: Hogwild user rows)")
    ap.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                    help="sub-steps on alternating compute streams (MFConfig.overlap_substeps; auto: from 4 ranks)")
    a = ap.parse_args()
    ws = [int(x) for x in a.ws.split(",")]
    if len(ws) > 1:  # one fresh child per world size (module docstring); the parent never touches the GPU
        import subprocess

        base = None
        for W in ws:
            argv = [sys.executable, os.path.abspath(__file__)] + [x for x in _argv_without_ws(sys.argv[1:])] + \
                ["--ws", str(W)]
            r = subprocess.run(argv, stdout=subprocess.PIPE, text=True)
            if r.returncode != 0:
                sys.exit(r.returncode)
            for line in r.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    base = base or d["ms_per_step"]
                    d["ratio_to_n1"] = d["ms_per_step"] / base  # to the first N of the list, as before
                    line = json.dumps(d)
                print(line, flush=True)
        return

    import torch

    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    dev = torch.device("cuda", 0)
    comm = Comm(device=dev)
    base = None
    for W in [int(x) for x in a.ws.split(",")]:
        cfg = MFConfig(num_users=a.users, num_items=a.items, dim=a.dim, learning_rate=0.01,
                       exchange="local" if W == 1 else "rotate", rotation=a.rotation, emulate_world=W if W > 1 else 0,
                       emulate_link_gbps=a.link_gbps, emulate_latency_us=a.latency_us,
                       overlap_substeps={"auto": "auto", "on": True, "off": False}[a.overlap],
                       user_update=a.user_update)
        m = DistributedMF(cfg, comm)
        data = SyntheticRatings(a.users, a.items, a.batch * a.pool, 0, W, device=dev)
        s = 0
        for _ in range(a.warmup):
            m.step(*data.batch(s, a.batch))
            s += 1
        m.flush()
        torch.cuda.synchronize()
        if W > 1:
            m.rot.wait_ms()  # drop the warm-up's waits
        t0 = time.perf_counter()
        for _ in range(a.steps):
            m.step(*data.batch(s, a.batch))
            s += 1
        m.flush()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        wait = m.rot.wait_ms() / a.steps if W > 1 else 0.0
        base = base or ms
        print(json.dumps({"emulated_world": W, "rotation": a.rotation if W > 1 else "local", "ms_per_step": ms,
                          "updates_per_s_per_gpu": a.batch / ms * 1e3, "ratio_to_n1": ms / base,
                          "users_per_gpu": m.users.n_local, "sub_steps": m.rot.K if W > 1 else 1,
                          "tile_rows": getattr(m, "tile_R", None), "tiles_per_block": getattr(m, "tile_T", None),
                          "user_phases": getattr(m, "user_phases", None), "user_update": m.user_update,
                          "link_gbps": a.link_gbps if W > 1 else None, "latency_us": a.latency_us if W > 1 else None,
                          "comm_wait_ms_per_step": wait, "exposed_fraction": wait / ms,
                          "overlap_substeps": bool(getattr(m, "_overlap", False)),
                          "link_bytes_per_step": (m.rot.bytes_sent / (a.steps + a.warmup)) if W > 1 else 0}),
              flush=True)
        if W > 1:
            m.rot.close()
        del m, data
        torch.cuda.empty_cache()


def _argv_without_ws(argv):
    out, skip = [], False
    for x in argv:
        if skip:
            skip = False
            continue
        if x == "--ws":
            skip = True
            continue
        if x.startswith("--ws="):
            continue
        out.append(x)
    return out


if __name__ == "__main__":
    main()
