#!/bin/bash
# GPU: partition tests; A/B partition levels x prefetch; clean profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py -q -x > gpurun_out/gpu_kt.log 2>&1; rc=$?
echo "kernel tests rc=$rc" >> gpurun_out/gpu_kt.log
tail -4 gpurun_out/gpu_kt.log
case $rc in 0) ;; *) echo "stopping after test rc=$rc"; exit 1;; esac
for L in 1 2; do
  FPS_TILE_PARTITION_LEVELS=$L timeout -k 10 300 python bench.py --steps 20 > gpurun_out/b_L${L}_pf.log 2>&1 || exit 1
  FPS_TILE_PARTITION_LEVELS=$L timeout -k 10 300 python bench.py --steps 20 --no-prefetch > gpurun_out/b_L${L}_nopf.log 2>&1 || exit 1
  echo "levels=$L prefetch: $(tail -1 gpurun_out/b_L${L}_pf.log | cut -c60-115)  no-prefetch: $(tail -1 gpurun_out/b_L${L}_nopf.log | cut -c60-115)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/L2nopf -- python bench.py --steps 5 --warmup 1 --no-prefetch > gpurun_out/prof_L2.log 2>&1 || exit 1
FPS_TILE_PARTITION_LEVELS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/L1nopf -- python bench.py --steps 5 --warmup 1 --no-prefetch > gpurun_out/prof_L1.log 2>&1 || exit 1
echo ALLDONE
