#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py tests/test_multirank_gpu.py -q -x -m gpu > gpurun_out/gpu_y.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_y.log
tail -4 gpurun_out/gpu_y.log
case $rc in 0) ;; *) echo "stopping after test rc=$rc"; exit 1;; esac
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/b_rec8_$i.log 2>&1 || exit 1
tail -1 gpurun_out/b_rec8_$i.log | cut -c1-160
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/rec8 -- python bench.py --steps 5 --warmup 1 --no-prefetch > gpurun_out/prof_rec8.log 2>&1 || exit 1
echo ALLDONE
