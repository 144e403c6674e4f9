#!/bin/bash
# A/B of the host early-exit test of the fused top-K scan (one sync per FPS_TOPK_BREAK_CHECK
# segments; 0 = never, the device LEMP skip alone), both top-K benches, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/brk
for rep in 1 2; do
  for v in 0 2 4 8; do
    FPS_TOPK_BREAK_CHECK=$v timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/brk/topk_$v.$rep.json 2>/dev/null || exit 1
    FPS_TOPK_BREAK_CHECK=$v timeout -k 10 300 python -u bench/bench_mf_topk.py > gpurun_out/brk/mftopk_$v.$rep.json 2>/dev/null || exit 1
    echo "break_check=$v rep$rep topk $(cut -d, -f2 gpurun_out/brk/topk_$v.$rep.json) mftopk $(cut -d, -f2 gpurun_out/brk/mftopk_$v.$rep.json)"
  done
done
