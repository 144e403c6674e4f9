#!/usr/bin/env python3
"""BASELINE config #3: word2vec skip-gram negative sampling, 1M vocab, dim 300, PS-sharded.

    python bench/bench_w2v.py [--gpus N] [--steps K] [--warmup W] [--pairs P]
    (N > 1 under torch.distributed.run: one PS shard per GPU, RCCL all-to-all)

Reports (center, context) pair-updates/s for the whole job: each pair updates
one input row and 1 + ``negatives`` output rows (block-shared negatives, MFMA
kernel, see csrc/kernels/sgns.hip).  Synthetic Zipf topic corpus, random init.
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
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=300)
    ap.add_argument("--pairs", type=int, default=1 << 20, help="pairs per GPU per step")
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--lr", type=float, default=0.005)
    ap.add_argument("--wire", default=None, choices=["fp32", "bf16"],
                    help="PS-path row dtype on the wire (pulled rows and pushed deltas; the owner accumulates in "
                         "fp32).  Default: bf16 at N > 1 -- dim-300 rows make the all-to-alls link-bound "
                         "(profiles/r5_ps_paths_emulated.md) -- fp32 at N = 1")
    ap.add_argument("--neg-group", type=int, default=None, choices=[1, 2, 4],
                    help="32-pair blocks sharing one set of negatives (default: SGNSConfig)")
    ap.add_argument("--ps-path", action="store_true",
                    help="N = 1: run the pull / push protocol instead of updating the tables in place")
    ap.add_argument("--shared-negatives", type=int, default=16, choices=[16, 32],
                    help="mode shared: negatives shared by each block of 32 pairs (16: kernel v4, 32: kernel v3)")
    ap.add_argument("--mode", default="standard", choices=["standard", "shared"],
                    help="standard: 5 independent negatives per pair (word2vec's objective, the reported number); "
                         "shared: block-shared negatives (Ji et al.), a different estimator")
    ap.add_argument("--negatives", type=int, default=5)
    ap.add_argument("--no-fuse-local-push", action="store_true",
                    help="PS path at one rank: push delta buffers and apply them (default: the kernel adds its "
                         "pushes into the owner's tables)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="N > 1: run rank 0 of an N-rank PS job on this one GPU under rank symmetry "
                         "(parallel/emulated.py: every all-to-all answered by this rank's own send buffer, "
                         "transfers modelled on device-timed links); reports the per-GPU rate at N")
    ap.add_argument("--emulate-mode", default="hot", choices=["hot", "symmetric"],
                    help="--emulate-world: 'hot' = the emulated rank is an OWNER as every peer sees it (it receives "
                         "from every peer what it sends itself: the skewed shard's real load); 'symmetric' = every "
                         "all-to-all answered by this rank's own send buffer (round 5)")
    ap.add_argument("--emulate-rank", type=int, default=-1,
                    help="--emulate-world: the rank to emulate (-1: the shard owning the most de-duplicated keys of "
                         "the first batch -- the owner the job waits for)")
    ap.add_argument("--link-gbps", type=float, default=50.0, help="--emulate-world: per-peer link rate (GB/s)")
    ap.add_argument("--latency-us", type=float, default=5.0, help="--emulate-world: per-message link latency")
    a = ap.parse_args(argv)

    import torch

    from flink_parameter_server_1_amd.models.w2v.sgns import DistributedSGNS, SGNSConfig, skipgram_pairs, \
        synthetic_corpus
    from flink_parameter_server_1_amd.parallel.comm import Comm

    shares = None
    if a.emulate_world > 1:
        from flink_parameter_server_1_amd.core.partitioners import HashPartitioner
        from flink_parameter_server_1_amd.parallel.emulated import SymmetricComm, shard_shares

        edev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        # both tables are hash-sharded: each shard's share of one micro-batch's distinct
        # center words (ranks draw alike)
        t0_ = synthetic_corpus(max(a.pairs // a.window, 1 << 16), a.vocab, seed=0, device=edev)
        shares = shard_shares(t0_[: a.pairs], HashPartitioner(a.emulate_world))
        if a.emulate_rank < 0:
            a.emulate_rank = max(range(a.emulate_world), key=lambda j: shares[j])
        comm = SymmetricComm(a.emulate_world, device=edev, link_gbps=a.link_gbps, latency_us=a.latency_us,
                             hot_owner=a.emulate_mode == "hot", rank=a.emulate_rank)
    else:
        comm = Comm.init_from_env()
    dev = comm.device
    if a.wire is None:
        a.wire = "bf16" if comm.world > 1 else "fp32"
    m = DistributedSGNS(SGNSConfig(vocab_size=a.vocab, dim=a.dim, window=a.window, learning_rate=a.lr,
                                   wire_dtype=a.wire, shared_negatives=a.shared_negatives,
                                   local_direct=not a.ps_path, mode=a.mode, negatives=a.negatives,
                                   fuse_local_push=not a.no_fuse_local_push,
                                   **({} if a.neg_group is None else {"neg_group": a.neg_group})), comm=comm)
    toks = synthetic_corpus(max(a.pairs // a.window, 1 << 16) * 2, a.vocab, seed=comm.rank, device=dev)
    c, o = skipgram_pairs(toks, a.window)
    n = c.numel()

    def batch(i):
        s = (i * a.pairs) % max(n - a.pairs, 1)
        return c[s:s + a.pairs], o[s:s + a.pairs]

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    loss0 = m.step(*batch(0), with_loss=True)
    for i in range(a.warmup):
        m.step(*batch(i + 1))
    m.flush()
    comm.barrier()
    sync()
    emu = a.emulate_world > 1
    if emu and dev.type == "cuda":
        comm.wait_ms()  # drop the warm-up's waits
    t0 = time.perf_counter()
    for i in range(a.steps):
        m.step(*batch(i + 1 + a.warmup))
    m.flush()  # the last batch's step and pushes run inside the timed region
    sync()
    comm.barrier()
    dt = comm.max_over_ranks(time.perf_counter() - t0)
    wait_ms = comm.wait_ms() / a.steps if emu and dev.type == "cuda" else 0.0
    loss1 = m.step(*batch(0), with_loss=True)
    if comm.rank == 0 or emu:
        # emulated: ONE GPU's rate at N is the measured value; N x it is a projection
        total = a.pairs * a.steps * (1 if emu else comm.world)
        per_gpu = a.pairs * a.steps / dt
        print(json.dumps({
            "metric": "word2vec SGNS pair-updates/sec per GPU (emulated N-rank job, hottest owner)" if emu else
                      "word2vec SGNS pair-updates/sec (whole node)",
            "value": total / dt, "unit": "pairs/s",
            "n_gpus": 1 if emu else comm.world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "dtype": "fp32",
            "emulated_world": a.emulate_world if emu else None,
            "emulate_mode": a.emulate_mode if emu else None, "emulated_rank": a.emulate_rank if emu else None,
            "shard_key_shares": shares,
            "projected_whole_node": {"value": per_gpu * a.emulate_world, "measured": False} if emu else None,
            "per_gpu_rate": per_gpu,
            "exposed_wait_ms_per_step": wait_ms if emu else None,
            "link_gbps": a.link_gbps if emu else None,
            "data": "synthetic Zipf topic corpus", "loss_first_last": [loss0, loss1],
            "config": {"model": f"sgns vocab={a.vocab} dim={a.dim} window={a.window} negatives={a.negatives}",
                       "mode": a.mode,
                       "negatives": (f"{a.negatives} independent per pair" if a.mode == "standard" else
                                     f"{a.shared_negatives} shared per {32 * m.cfg.neg_group} pairs, weight "
                                     f"{a.negatives}/{a.shared_negatives}"),
                       "exchange": "local-direct" if m._direct else "ps",
                       "fused_local_push": (not m._direct and m.cfg.fuse_local_push and comm.world == 1),
                       "pairs_per_gpu_step": a.pairs, "wire_dtype": a.wire},
        }), flush=True)
    comm.shutdown()  # every rank leaves the process group together


if __name__ == "__main__":
    main()
