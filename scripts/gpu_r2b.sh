#!/bin/bash
# Round 2 checkpoint: full GPU suite, smoke, bench, marker-trace profile (roctx ranges + kernels).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2b/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r2b/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b/smoke.log 2>&1 || { tail -20 gpurun_out/r2b/smoke.log; exit 1; }
tail -1 gpurun_out/r2b/smoke.log
timeout -k 10 300 python bench.py --metrics-jsonl gpurun_out/r2b/bench_metrics.jsonl > gpurun_out/r2b/bench.log 2>&1 || { tail -20 gpurun_out/r2b/bench.log; exit 1; }
tail -1 gpurun_out/r2b/bench.log | cut -c1-250
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/r2b/prof_marker -- python bench.py --steps 5 --warmup 2 > gpurun_out/r2b/prof_marker.log 2>&1 || { tail -20 gpurun_out/r2b/prof_marker.log; exit 1; }
echo ALLDONE
