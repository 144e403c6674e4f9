#!/bin/bash
# Both item blocks of a user phase in one tiled-SGD launch: numerics + A/B on the headline bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pair
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py -m gpu -k "tiled" -x -q --timeout 120 --timeout-method thread > gpurun_out/pair/tests.log 2>&1 || { tail -30 gpurun_out/pair/tests.log; exit 1; }
tail -1 gpurun_out/pair/tests.log
for rep in 1 2; do
for M in 0 1; do
  FPS_MF_PAIR=$M timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/pair/b_$M.log 2>&1 || { tail -20 gpurun_out/pair/b_$M.log; exit 1; }
  echo "pair=$M $(grep '^{' gpurun_out/pair/b_$M.log | cut -c80-200)"
done
done
FPS_MF_PAIR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pair/prof -- python bench.py --steps 5 --warmup 1 --no-prefetch > gpurun_out/pair/prof.log 2>&1 || exit 1
echo ALLDONE
