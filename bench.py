#!/usr/bin/env python3
"""Headline benchmark: MF-SGD param updates/s, 10M users x 1M items, rank 64.

Metric and config from BASELINE.json: "param updates/sec (whole node), MF-SGD
10M x 1M rank-64 at 1/2/4/8 MI355X".  One update = one rating-SGD step
(one user row + one item row of 64 fp32 each).  Synthetic ratings, random
init, fp32 parameters and compute.

At N > 1 the default exchange is the item-block ring rotation
(``--exchange rotate``, ``parallel/rotation.py``): the 1M x 64 item table
travels around the xGMI ring in 2N blocks while every GPU updates the block it
holds with its users' ratings -- each item block is owned by one GPU at a time,
so the updates are exact (no staleness) and each block transfer (256 MB / 2N)
hides behind the compute of the resident block.  The SGD kernel is the
tile-grouped one (``csrc/kernels/mf_tiled.hip``: ratings bucketed by item
tile, one lane group per item row, no item atomics).  ``--exchange ps`` runs the
reference's pull/push protocol instead (dedup -> all-to-all pull -> SGD ->
all-to-all push; rows cross xGMI as fp32, ``--wire bf16`` halves the bytes; the
pull of micro-batch k+1 overlaps the SGD of k, ``--no-pipeline`` disables it).

    python bench.py --gpus N --steps K --warmup W
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Weak scaling: every GPU processes ``--batch`` ratings per step (its users'
ratings, as ``psOnlineMF`` partitions input by ``user % W``); value = total
updates/s over all GPUs, timed between barriers + device syncs, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch_guard(argv) -> None:
    """``--gpus N`` (N > 1) must run N ranks.  Without torchrun env vars the
    launcher is started as a CHILD process (nothing GPU-related has been loaded
    in this parent: torch is not imported yet) and this process exits with its
    code; under torchrun a WORLD_SIZE that disagrees with ``--gpus`` is an error.
    A mis-launched scaling run can therefore never report N = 1 numbers as N."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args(argv)
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if a.gpus > 1:
            import subprocess

            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
                   "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
            cmd += list(argv)
            print(f"[bench] --gpus {a.gpus} without torchrun: launching {a.gpus} ranks", file=sys.stderr, flush=True)
            sys.exit(subprocess.call(cmd))
        return
    if int(world) != a.gpus:
        print(f"[bench] error: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
        sys.exit(2)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    _launch_guard(argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 26,
                    help="ratings per GPU per step.  At N > 1 every GPU receives the whole item table (256 MB) "
                         "once per step around the ring (~5 ms at ~50 GB/s per xGMI link); 64M ratings (~9 ms of "
                         "SGD) keep the transfers hidden behind the compute")
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--pool", type=int, default=4, help="data pool = pool * batch ratings per GPU")
    ap.add_argument("--exchange", default="auto", choices=["auto", "rotate", "ps", "local"],
                    help="auto = local at N=1, rotate at N>1")
    ap.add_argument("--rotation", default="bidir", choices=["bidir", "ring"],
                    help="rotate: two counter-rotating rings of quarter-shard blocks (both directions of two xGMI "
                         "links) or one ring of half-shard blocks")
    ap.add_argument("--wire", default="fp32", choices=["fp32", "bf16"],
                    help="PS-path all-to-all row dtype (bf16 halves the bytes; opt-in: the headline keeps fp32)")
    ap.add_argument("--no-pipeline", action="store_true")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="tiled SGD: partition each batch on the main stream instead of prefetching it")
    ap.add_argument("--user-update", default="auto", choices=["auto", "store", "sc1", "atomic"],
                    help="store: Hogwild user rows (plain accesses); sc1: write-through user rows (about half the lost "
                         "user updates); atomic: exact -- the tiled kernel adds every user delta with float atomics "
                         "(none lost, ~2x the step: float atomics run at ~1.29 TB/s at every working set, "
                         "profiles/r6_exact_user_rows.md); auto (default): store at every N -- one semantics for "
                         "the whole scaling curve; the exact mode is timed beside it (--exact-steps)")
    ap.add_argument("--exact-steps", type=int, default=5,
                    help="after the timed loop, time this many steps of the exact user-row mode (atomic) on the same "
                         "model and report exact_updates_per_s / exact_ms_per_step (0 = skip; tiled SGD only)")
    ap.add_argument("--sgd-mode", default="auto", choices=["auto", "tiled", "grouped", "flat"],
                    help="auto = tiled (tile-grouped kernel, no item atomics) where it applies")
    ap.add_argument("--user-phases", type=int, default=0,
                    help="tiled SGD: user-range phases per step (0 = auto, ~2.5M users per phase)")
    ap.add_argument("--force-ps-path", action="store_true",
                    help="run dedup/pull/push even at N=1 (measures the N>1 step minus RCCL)")
    ap.add_argument("--no-fuse-local-push", action="store_true",
                    help="--force-ps-path at N=1: push the delta buffer through the PS apply instead of letting the "
                         "tiled kernel update the served shard in place")
    ap.add_argument("--watchdog-s", type=float, default=0.0,
                    help="fail fast: end this rank (exit 17) when a step makes no progress for this long (0 = off)")
    ap.add_argument("--no-hogwild-probe", action="store_true",
                    help="skip the side probe of lost user updates (run after the timed loop, reported in config)")
    ap.add_argument("--verify", dest="verify", action="store_true", default=None,
                    help="before timing, run a small instance of this exchange on the real process group and compare "
                         "it with a sequential CPU replay (parallel/verify.py); a mismatch exits non-zero before any "
                         "value is printed.  Default: on at N > 1")
    ap.add_argument("--no-verify", dest="verify", action="store_false")
    ap.add_argument("--metrics-jsonl", default=None,
                    help="append per-step stage timings (HIP events) and counters of rank 0 to this JSON-lines file")
    a = ap.parse_args(argv)

    import torch

    from flink_parameter_server_1_amd import ops
    from flink_parameter_server_1_amd.models.mf.fast import DistributedMF, MFConfig, SyntheticRatings
    from flink_parameter_server_1_amd.parallel.comm import Comm

    comm = Comm.init_from_env()
    if comm.device.type == "cuda" and not ops.native_available():
        raise RuntimeError("gfx950 kernel library not built: run python csrc/build.py")
    dev = comm.device
    n = comm.world
    if a.gpus != n:  # unreachable after _launch_guard; kept as a hard invariant
        raise SystemExit(f"[bench] --gpus {a.gpus} but the process group has {n} ranks")
    verify = None
    if a.verify if a.verify is not None else n > 1:
        # the exchange of THIS job on THIS process group against a sequential replay,
        # before anything is timed; every rank learns the verdict and exits on a mismatch
        import torch.distributed as dist
        from flink_parameter_server_1_amd.parallel import verify as V

        # the exchange MFConfig picks for this job (force_ps_path -> the PS protocol)
        ex = a.exchange if a.exchange in ("rotate", "ps") else \
            ("ps" if a.force_ps_path else ("rotate" if n > 1 else "local"))
        if ex == "local":
            ex = "rotate"  # world 1: the rotation path without peers
        mut = os.environ.get("FPS_VERIFY_MUTANT")  # fault injection: the check's own tests
        verify = V.rotation_check(comm, schedule=a.rotation, exchange=ex, pipeline=not a.no_pipeline, wire=a.wire,
                                  rotation_cls=V.mutant_rotation(mut) if mut else None, user_update=a.user_update,
                                  sgd_mode=a.sgd_mode, dim=a.dim)
        if verify["verify_ok"] and ex == "rotate" and (a.user_update == "atomic" or a.exact_steps > 0):
            # the exact user-row mode this job times, in the collision regime (users repeated
            # 8 times per step, under the real rotation and sub-step overlap)
            col = V.rotation_check(comm, schedule=a.rotation, exchange=ex, user_update="atomic", sgd_mode=a.sgd_mode,
                                   dim=a.dim, repeated_users=True,
                                   rotation_cls=V.mutant_rotation(mut) if mut else None)
            verify["collision"] = col
            if a.user_update == "atomic":  # the timed mode itself: a failure ends the job
                verify["verify_ok"] = bool(col["verify_ok"])
            elif not col["verify_ok"]:  # only the side measurement's mode: it is not reported
                a.exact_steps = 0
        ids = [V.device_identity(comm)]
        if n > 1:
            ids = [None] * n
            dist.all_gather_object(ids, V.device_identity(comm))
        verify["devices"] = ids
        verify["rccl_version"] = V.rccl_version() if comm.device.type == "cuda" else None
        if comm.backend == "nccl":  # one GPU per rank: a shared device would make the check meaningless
            uu = [d.get("uuid") or d.get("device") for d in ids]
            if len(set(uu)) != n:
                verify["verify_ok"] = False
                verify["verify_error"] = f"ranks share devices: {uu}"
        if not verify["verify_ok"]:
            if comm.rank == 0:
                print(f"[bench] VERIFY FAILED: {json.dumps(verify)}", file=sys.stderr, flush=True)
            sys.exit(3)
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    cfg = MFConfig(num_users=a.users, num_items=a.items, dim=a.dim, learning_rate=a.lr, wire_dtype=a.wire,
                   user_update=a.user_update, force_ps_path=a.force_ps_path, sgd_mode=a.sgd_mode,
                   pipeline=not a.no_pipeline, exchange=a.exchange, prefetch_partition=not a.no_prefetch,
                   user_phases=a.user_phases, rotation=a.rotation, fuse_local_push=not a.no_fuse_local_push)
    model = DistributedMF(cfg, comm)
    data = SyntheticRatings(a.users, a.items, a.batch * a.pool, comm.rank, n, device=comm.device)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    timer = None
    if a.metrics_jsonl:
        from flink_parameter_server_1_amd.utils.metrics import StageTimer

        timer = StageTimer(device=dev.type == "cuda")
    wd = None
    if a.watchdog_s > 0:
        from flink_parameter_server_1_amd.utils.watchdog import Watchdog

        wd = Watchdog(a.watchdog_s, name=f"bench rank {comm.rank}").start()
    step = 0
    for _ in range(a.warmup):
        model.step(*data.batch(step, a.batch))
        step += 1
        if wd is not None:
            wd.beat(step)
    model.flush()
    comm.barrier()
    sync()
    model.set_timer(timer)  # None unless --metrics-jsonl: event records only, no syncs
    if model.exchange == "rotate":
        model.rot.wait_ms()  # drop the warm-up's transfer waits
    t0 = time.perf_counter()
    for _ in range(a.steps):
        model.step(*data.batch(step, a.batch))
        step += 1
        if wd is not None:
            wd.beat(step)
        if timer is not None:
            timer.step_end()
    model.flush()  # the last micro-batch's SGD + push run inside the timed region
    sync()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt_max = comm.max_over_ranks(dt)
    # time the compute stream waited for rotation transfers (HIP events around each
    # wait; read after the timed region): "transfer exposed" vs "compute slower"
    wait_ms = model.rot.wait_ms() / a.steps if model.exchange == "rotate" else 0.0
    waits = comm.gather_floats(wait_ms)
    n_local = comm.gather_floats(float(model.users.n_local))
    # per-rank bytes this rank put on the wire (all-to-all + ring rotation)
    sent = float(comm.bytes_sent + (model.rot.bytes_sent if model.exchange == "rotate" else 0))
    bytes_per_rank = comm.gather_floats(sent)
    import torch.distributed as dist

    # the exact user-row mode on the same model, data and schedule (outside the headline's
    # timed region, timed the same way): every rating's user delta added with float atomics
    exact = None
    if a.exact_steps > 0 and model.sgd_mode == "tiled" and model.user_update != "atomic" and dev.type == "cuda":
        mode0 = model.user_update
        model.set_user_update("atomic")
        model.step(*data.batch(step, a.batch))  # one untimed step in the mode
        step += 1
        model.flush()
        sync()
        comm.barrier()
        sync()
        t1 = time.perf_counter()
        for _ in range(a.exact_steps):
            model.step(*data.batch(step, a.batch))
            step += 1
        model.flush()
        sync()
        comm.barrier()
        sync()
        dte = comm.max_over_ranks(time.perf_counter() - t1)
        model.set_user_update(mode0)
        exact = {"exact_updates_per_s": a.batch * a.exact_steps * n / dte, "exact_ms_per_step": dte / a.exact_steps * 1e3,
                 "exact_steps": a.exact_steps}
    elif model.user_update == "atomic":
        exact = {"exact_updates_per_s": a.batch * a.steps * n / dt_max, "exact_ms_per_step": dt_max / a.steps * 1e3,
                 "exact_steps": a.steps}

    # side probe (outside the timed region): the Hogwild user-row race of the tiled SGD
    # measured on this rank's geometry -- users per GPU, the same batch and user phases
    # (bench/probe_hogwild.py: user rows from 0, tiny step, every lost contribution
    # counted by least squares per user); rank 0 only, the others wait at the barrier
    hog = None
    if (not a.no_hogwild_probe and dev.type == "cuda" and model.sgd_mode == "tiled" and model.exchange != "ps"
            and comm.rank == 0):
        sys.path.insert(0, os.path.join(ROOT, "bench"))
        from probe_hogwild import lost_updates

        del data
        torch.cuda.empty_cache()
        n_loc = model.users.n_local
        try:  # a side measurement: its failure must not cost the timed result
            hog = lost_updates(n_loc, a.items, a.batch / n_loc, getattr(model, "user_phases", 1),
                               user_update=model.user_update, world=n if model.exchange == "rotate" else 1)
        except Exception as e:  # noqa: BLE001 -- reported, the bench line still prints
            print(f"hogwild side probe failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
            hog = None
        torch.cuda.empty_cache()
    comm.barrier()

    world_seen = dist.get_world_size() if dist.is_initialized() else 1
    backend = dist.get_backend() if dist.is_initialized() else "none (single process)"
    total_updates = a.batch * a.steps * n
    value = total_updates / dt_max
    if comm.rank == 0:
        out = {
            "metric": "param updates/sec (whole node), MF-SGD 10Mx1M rank-64",
            "value": value,
            "unit": "updates/s",
            "n_gpus": n,
            "world_size": world_seen,
            "backend": backend,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt_max / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (uniform users/items, U[0,1) ratings; random-init U[-0.01,0.01) factors)",
            "config": {
                "model": f"mf-sgd users={a.users} items={a.items} rank={a.dim}",
                "global_batch": a.batch * n,
                "seq_len": None,
                "parallelism": f"dp{n} (users by user%W) + ps{n} (items hash-sharded, exchange={model.exchange})",
                "exchange": model.exchange,
                "fuse_local_push": cfg.fuse_local_push if model.exchange == "ps" else None,
                "wire_dtype": a.wire if model.exchange == "ps" else "none (fp32 parameters stay resident or travel "
                                                                     "whole)",
                "sgd_mode": model.sgd_mode,
                "user_phases": getattr(model, "user_phases", None),
                "pipelined": model.pipeline,
                "scalar_params_per_s": value * 2 * a.dim,
                "unique_items_per_step_per_gpu": (model.ps.stats["unique"] / max(model.ps.stats["steps"], 1))
                if model.exchange == "ps" else None,
                "rotation": model.cfg.rotation if model.exchange == "rotate" else None,
                "overlap_substeps": bool(getattr(model, "_overlap", False)),
                "rotation_bytes_sent_rank0": model.rot.bytes_sent if model.exchange == "rotate" else None,
                "comm_wait_ms_per_step": max(waits),
                "comm_wait_ms_per_step_per_rank": waits,
                "users_per_rank": [int(x) for x in n_local],
                "bytes_sent_per_rank": bytes_per_rank,
                "bytes_per_peer_rank0": list(comm.peer_bytes),
                "user_update": model.user_update,
                # Hogwild race of the user rows (side probe on rank 0's geometry, not timed):
                # fraction of rated users that lost >= 1 update, fraction of rating updates lost
                "lost_user_fraction": None if hog is None else hog["lost_user_fraction"],
                "lost_user_update_fraction": None if hog is None else hog.get("lost_update_fraction"),
            },
        }
        lf = out["config"]["lost_user_update_fraction"]
        # updates that survive the Hogwild user-row race (value counts every rating's update;
        # user_update="atomic" loses none): value x (1 - lost fraction), None when unmeasured
        out["effective_updates_per_s"] = value * (1.0 - lf) if lf is not None else \
            (value if model.user_update == "atomic" else None)
        if exact is not None:  # the exact mode (0 lost user updates), timed on the same job
            out.update(exact)
        if verify is not None:
            out["verify_ok"] = verify["verify_ok"]
            out["verify"] = verify
        print(json.dumps(out), flush=True)
    if timer is not None:
        timer.step_end()  # the flush's stages
        steps_ms = timer.per_step_ms()
        if comm.rank == 0:
            from flink_parameter_server_1_amd.utils.metrics import JsonlWriter

            w = JsonlWriter(a.metrics_jsonl)
            for i, st in enumerate(steps_ms):
                w.write(kind="step", step=i, stage_ms=st)
            w.write(kind="summary", ms_per_step=dt_max / a.steps * 1e3, counters=model.metrics(), n_gpus=n)
            w.close()
    if wd is not None:
        wd.stop()
    if n > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
