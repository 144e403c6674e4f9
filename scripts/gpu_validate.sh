#!/bin/bash
# Full GPU validation on one MI355X: gpu test suite, smoke(), headline bench, kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.log 2>&1 || { tail -20 gpurun_out/bench_n1.log; exit 1; }
tail -1 gpurun_out/bench_n1.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/bench -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_bench.log 2>&1 || exit 1
echo ALLDONE
