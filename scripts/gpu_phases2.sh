#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ph2
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "tile_partition" -x -q --timeout 120 --timeout-method thread > gpurun_out/ph2/tests.log 2>&1 || { tail -30 gpurun_out/ph2/tests.log; exit 1; }
tail -1 gpurun_out/ph2/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ph2/bench.log 2>&1 || { tail -20 gpurun_out/ph2/bench.log; exit 1; }
echo "$(grep '^{' gpurun_out/ph2/bench.log | cut -c80-200)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ph2/prof -- python bench.py --steps 5 --warmup 1 --no-prefetch > gpurun_out/ph2/prof.log 2>&1 || exit 1
echo ALLDONE
