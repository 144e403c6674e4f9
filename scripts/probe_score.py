"""Time the fused top-K scorers on one 4096 x 65536 x 64 segment (thresholds from a
real seed segment, so few scores pass): without / with the per-tile LEMP bound."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from flink_parameter_server_1_amd import ops


def main():
    B, n, D, k = int(os.environ.get("PB", 4096)), 65536, 64, 75
    g = torch.Generator(device="cuda").manual_seed(0)
    Q = (torch.rand(B, D, generator=g, device="cuda") * 0.2 - 0.1)
    X = (torch.rand(n + 4096, D, generator=g, device="cuda") * 0.2 - 0.1)
    ids = torch.arange(n + 4096, device="cuda")
    best_s = torch.full((B, k), float("-inf"), device="cuda")
    best_i = torch.full((B, k), -1, dtype=torch.long, device="cuda")
    ops.topk_merge(ops.score_gemm(Q, X[:4096]), ids[:4096], best_s, best_i)
    cap = 2048
    ck = torch.empty((B, cap), dtype=torch.int32, device="cuda")
    ci = torch.empty((B, cap), dtype=torch.long, device="cuda")
    cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
    X1, I1 = X[4096:4096 + n // 2].contiguous(), ids[4096:4096 + n // 2].contiguous()
    Xs, I = X[4096 + n // 2:].contiguous(), ids[4096 + n // 2:].contiguous()
    dense = best_s.clone()
    # steady state: thresholds after merging another half segment
    cnt.zero_()
    ops.score_filter(Q, X1, I1, best_s, ck, ci, cnt)
    ops.topk_merge_cand(ck, ci, cnt, best_s, best_i)
    steady = best_s.clone()
    none = torch.full_like(best_s, 1e30)
    ql = torch.linalg.vector_norm(Q, dim=1)
    xl = torch.linalg.vector_norm(Xs, dim=1)
    nn = Xs.shape[0]
    res = {}
    for tname, th in (("dense", dense), ("steady", steady), ("none", none)):
        variants = {
            "tile64": lambda: ops.score_filter(Q, Xs, I, th, ck, ci, cnt),
            "lemp_nolen": lambda: ops.score_filter_lemp(Q, Xs, I, th, ck, ci, cnt),
            "lemp_len": lambda: ops.score_filter_lemp(Q, Xs, I, th, ck, ci, cnt, ql, xl),
        }
        if tname == "none":
            variants["gemm64"] = lambda: ops.score_gemm(Q, Xs)
        for name, fn in variants.items():
            for _ in range(3):
                cnt.zero_(); fn()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            reps = 20
            t = 0.0
            for _ in range(reps):
                cnt.zero_()
                ev[0].record(); fn(); ev[1].record()
                torch.cuda.synchronize()
                t += ev[0].elapsed_time(ev[1])
            us = t / reps * 1e3
            res[f"{tname}.{name}"] = {"us": round(us, 1), "tflops": round(2 * B * nn * D / us / 1e6, 1),
                                      "passed_per_q": round(int(cnt.sum()) / B, 1)}
    print(json.dumps(res, indent=0))


if __name__ == "__main__":
    main()
