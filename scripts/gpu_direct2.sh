#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/d2
timeout -k 10 300 python -u -m pytest tests/test_pa_fast.py tests/test_sgns_sampling.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/d2/tests.log 2>&1 || { tail -30 gpurun_out/d2/tests.log; exit 1; }
tail -1 gpurun_out/d2/tests.log
timeout -k 10 300 python bench/bench_pa.py > gpurun_out/d2/pa.log 2>&1 || { tail -20 gpurun_out/d2/pa.log; exit 1; }
grep '^{' gpurun_out/d2/pa.log | cut -c1-200
timeout -k 10 300 python bench/bench_w2v.py > gpurun_out/d2/w2v.log 2>&1 || { tail -20 gpurun_out/d2/w2v.log; exit 1; }
grep '^{' gpurun_out/d2/w2v.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/d2/prof -- python bench/bench_pa.py --steps 8 --warmup 2 > gpurun_out/d2/prof.log 2>&1 || exit 1
echo ALLDONE
