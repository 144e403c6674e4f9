#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w2vd
timeout -k 10 300 python -u -m pytest tests/test_sgns_sampling.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/w2vd/tests.log 2>&1 || { tail -30 gpurun_out/w2vd/tests.log; exit 1; }
tail -1 gpurun_out/w2vd/tests.log
timeout -k 10 300 python bench/bench_w2v.py > gpurun_out/w2vd/bench.log 2>&1 || { tail -20 gpurun_out/w2vd/bench.log; exit 1; }
grep '^{' gpurun_out/w2vd/bench.log | cut -c1-420
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w2vd/prof -- python bench/bench_w2v.py --steps 8 --warmup 2 > gpurun_out/w2vd/prof.log 2>&1 || exit 1
echo ALLDONE
