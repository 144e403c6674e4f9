#!/usr/bin/env python3
"""SGNS kernel alone (K6): v3 / v4 on the same pulled rows, timed with HIP events.

    python bench/bench_sgns_kernel.py [--pairs 1048576] [--dim 300]

Inputs mimic one bench_w2v step: center-major pairs over a Zipf corpus, rows
pulled (deduplicated) into compact in/out tables, 16 (or 32) shared negatives per
block of 32 pairs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1 << 20)
    ap.add_argument("--dim", type=int, default=300)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args(argv)

    import torch

    from flink_parameter_server_1_amd import ops
    from flink_parameter_server_1_amd.models.w2v.sgns import skipgram_pairs, synthetic_corpus

    dev = torch.device("cuda", 0)
    toks = synthetic_corpus(max(a.pairs // 5, 1 << 16) * 2, a.vocab, seed=0, device=dev)
    c, o = skipgram_pairs(toks, 5)
    c, o = c[:a.pairs].contiguous(), o[:a.pairs].contiguous()
    P = c.numel()
    uc, pos_c = torch.unique(c, return_inverse=True)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    for neg_k, kernels in ((16, ("v4",)), (32, ("v3",))):
        nb = (P + 31) // 32
        negs = torch.randint(0, a.vocab, (nb * neg_k,), device=dev, generator=g, dtype=c.dtype)
        uo, inv = torch.unique(torch.cat([o, negs]), return_inverse=True)
        pos_o, pos_neg = inv[:P].int().contiguous(), inv[P:].int().contiguous()
        rows_in = (torch.rand(uc.numel(), a.dim, device=dev) - 0.5) / a.dim
        rows_out = (torch.rand(uo.numel(), a.dim, device=dev) - 0.5) / a.dim
        for kern in kernels:
            d_in = torch.zeros_like(rows_in)
            d_out = torch.zeros_like(rows_out)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ops.sgns_step(rows_in, rows_out, pos_c.int(), pos_o, pos_neg, 0.005, 5 / neg_k, d_in, d_out,
                          neg_k=neg_k)
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(a.reps):
                ev[0].record()
                ops.sgns_step(rows_in, rows_out, pos_c.int(), pos_o, pos_neg, 0.005, 5 / neg_k, d_in, d_out,
                              neg_k=neg_k)
                ev[1].record()
                torch.cuda.synchronize()
                best = min(best, ev[0].elapsed_time(ev[1]))
            print(json.dumps({"kernel": kern or "v3", "neg_k": neg_k, "pairs": P, "dim": a.dim, "ms": round(best, 3),
                              "pairs_per_s": P / best * 1e3, "unique_in": uc.numel(), "unique_out": uo.numel()}),
                  flush=True)


if __name__ == "__main__":
    main()
