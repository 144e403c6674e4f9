#!/bin/bash
# GPU pass: tiled MF kernel tests + benches + kernel profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/gpu_kt.log 2>&1; rc=$?
echo "kernel tests rc=$rc" >> gpurun_out/gpu_kt.log
tail -15 gpurun_out/gpu_kt.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py > gpurun_out/b_tiled.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --sgd-mode flat > gpurun_out/b_flat.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --exchange rotate > gpurun_out/b_rot_tiled.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --batch 4194304 > gpurun_out/b_tiled4m.log 2>&1 || exit 1
for f in b_tiled b_flat b_rot_tiled b_tiled4m; do tail -1 gpurun_out/$f.log | cut -c1-200; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/tiled -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_tiled.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/rot_tiled -- python bench.py --exchange rotate --steps 5 --warmup 1 > gpurun_out/prof_rot_tiled.log 2>&1 || exit 1
echo ALLDONE
