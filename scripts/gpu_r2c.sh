#!/bin/bash
# Round 2 checkpoint c: full GPU suite, smoke, bench, MF+top-K kernel profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2c/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r2c/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c/smoke.log 2>&1 || { tail -20 gpurun_out/r2c/smoke.log; exit 1; }
tail -1 gpurun_out/r2c/smoke.log
timeout -k 10 300 python bench.py --metrics-jsonl gpurun_out/r2c/bench_metrics.jsonl > gpurun_out/r2c/bench.log 2>&1 || { tail -20 gpurun_out/r2c/bench.log; exit 1; }
tail -1 gpurun_out/r2c/bench.log | cut -c1-250
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2c/prof_mftopk -- python bench/bench_mf_topk.py --steps 10 --warmup 2 > gpurun_out/r2c/prof_mftopk.log 2>&1 || { tail -20 gpurun_out/r2c/prof_mftopk.log; exit 1; }
echo ALLDONE
