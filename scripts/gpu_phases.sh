#!/bin/bash
# User phases in the tiled MF step: numerics, bench P=1 vs auto, kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ph
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py -k "phases" -x -q --timeout 120 --timeout-method thread > gpurun_out/ph/tests.log 2>&1 || { tail -30 gpurun_out/ph/tests.log; exit 1; }
tail -2 gpurun_out/ph/tests.log
for P in 1 0 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --user-phases $P > gpurun_out/ph/bench_P$P.log 2>&1 || { tail -20 gpurun_out/ph/bench_P$P.log; exit 1; }
  echo "P$P $(grep '^{' gpurun_out/ph/bench_P$P.log | cut -c80-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ph/prof -- python bench.py --steps 5 --warmup 1 > gpurun_out/ph/prof.log 2>&1 || exit 1
echo ALLDONE
