#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests/test_multirank_gpu.py tests/test_topk_fast.py -q -x -m gpu > gpurun_out/gpu_mr.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_mr.log
tail -15 gpurun_out/gpu_mr.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench/bench_topk.py > gpurun_out/b_topk3.log 2>&1 || exit 1
tail -1 gpurun_out/b_topk3.log | cut -c1-200
echo ALLDONE
