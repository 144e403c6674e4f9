#!/bin/bash
# Tiled SGD with the wave-parallel in-tile row scan: numerics + bench + kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scan
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py -m gpu -k "tiled" -x -q --timeout 120 --timeout-method thread > gpurun_out/scan/tests.log 2>&1 || { tail -30 gpurun_out/scan/tests.log; exit 1; }
tail -1 gpurun_out/scan/tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/scan/b.log 2>&1 || { tail -20 gpurun_out/scan/b.log; exit 1; }
  echo "$(grep '^{' gpurun_out/scan/b.log | cut -c80-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scan/prof -- python bench.py --steps 5 --warmup 1 --no-prefetch > gpurun_out/scan/prof.log 2>&1 || exit 1
echo ALLDONE
