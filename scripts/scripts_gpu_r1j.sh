#!/bin/bash
# GPU pass: tiled MF kernel v2 (packed records) tests + benches + profile + LDS counters.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/gpu_kt.log 2>&1; rc=$?
echo "kernel tests rc=$rc" >> gpurun_out/gpu_kt.log
tail -4 gpurun_out/gpu_kt.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py > gpurun_out/b_tiled.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --exchange rotate > gpurun_out/b_rot_tiled.log 2>&1 || exit 1
for f in b_tiled b_rot_tiled; do tail -1 gpurun_out/$f.log | cut -c1-200; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/tiled3 -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_tiled3.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/tiled3_pmc -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof_tiled3_pmc.log 2>&1
echo "pmc rc=$?"
echo ALLDONE
