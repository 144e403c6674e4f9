#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pad
timeout -k 10 300 python -u -m pytest tests/test_pa_fast.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pad/tests.log 2>&1 || { tail -30 gpurun_out/pad/tests.log; exit 1; }
tail -1 gpurun_out/pad/tests.log
timeout -k 10 300 python bench/bench_pa.py > gpurun_out/pad/bench.log 2>&1 || { tail -20 gpurun_out/pad/bench.log; exit 1; }
grep '^{' gpurun_out/pad/bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pad/prof -- python bench/bench_pa.py --steps 8 --warmup 2 > gpurun_out/pad/prof.log 2>&1 || exit 1
echo ALLDONE
