#!/bin/bash
# LDS-sorted two-level tile partition (levels=3): numerics, bench vs levels 1/2, kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tp3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "tile_partition or tiled" -x -q --timeout 120 --timeout-method thread > gpurun_out/tp3/tests.log 2>&1 || { tail -30 gpurun_out/tp3/tests.log; exit 1; }
tail -2 gpurun_out/tp3/tests.log
for L in 3; do
  FPS_TILE_PARTITION_LEVELS=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/tp3/bench_L$L.log 2>&1 || { tail -20 gpurun_out/tp3/bench_L$L.log; exit 1; }
  echo "L$L $(grep '^{' gpurun_out/tp3/bench_L$L.log | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp3/prof -- python bench.py --steps 5 --warmup 1 --no-prefetch > gpurun_out/tp3/prof.log 2>&1 || exit 1
timeout -k 10 300 python bench/bench_tiled_substeps.py > gpurun_out/tp3/substeps.log 2>&1 || { tail -20 gpurun_out/tp3/substeps.log; exit 1; }
grep '^{' gpurun_out/tp3/substeps.log
echo ALLDONE
