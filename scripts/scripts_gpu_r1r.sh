#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 300 python -m pytest tests/test_sgns_sampling.py -q -x -m gpu > gpurun_out/gpu_sgns.log 2>&1; rc=$?
echo "sgns tests rc=$rc" >> gpurun_out/gpu_sgns.log
tail -4 gpurun_out/gpu_sgns.log
case $rc in 0) ;; *) echo "stopping after test rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench/bench_w2v.py > gpurun_out/b_w2v3.log 2>&1 || exit 1
tail -1 gpurun_out/b_w2v3.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/w2v3 -- python bench/bench_w2v.py --steps 5 --warmup 1 > gpurun_out/prof_w2v3.log 2>&1 || exit 1
echo ALLDONE
