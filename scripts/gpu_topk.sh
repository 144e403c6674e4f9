#!/bin/bash
# Fused top-K scoring: numerics + bench_topk + kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/topk
timeout -k 10 300 python -u -m pytest tests/test_topk_fast.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/topk/tests.log 2>&1 || { tail -40 gpurun_out/topk/tests.log; exit 1; }
tail -1 gpurun_out/topk/tests.log
timeout -k 10 300 python bench/bench_topk.py > gpurun_out/topk/b.log 2>&1 || { tail -20 gpurun_out/topk/b.log; exit 1; }
grep '^{' gpurun_out/topk/b.log | cut -c1-330
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/topk/prof -- python bench/bench_topk.py --steps 5 --warmup 1 > gpurun_out/topk/prof.log 2>&1 || exit 1
echo ALLDONE
