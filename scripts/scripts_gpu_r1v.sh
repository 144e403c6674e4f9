#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -q -x -m gpu > gpurun_out/gpu_all.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_all.log
tail -5 gpurun_out/gpu_all.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench/bench_topk.py > gpurun_out/b_topk2.log 2>&1 || exit 1
tail -1 gpurun_out/b_topk2.log | cut -c1-400
timeout -k 10 300 python bench/bench_pa.py --steps 10 --warmup 2 > gpurun_out/b_pa5.log 2>&1 || exit 1
tail -1 gpurun_out/b_pa5.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/topk2 -- python bench/bench_topk.py --steps 5 --warmup 1 > gpurun_out/prof_topk2.log 2>&1 || exit 1
echo ALLDONE
