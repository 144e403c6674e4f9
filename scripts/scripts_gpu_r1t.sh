#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -q -x -m gpu > gpurun_out/gpu_all.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_all.log
tail -5 gpurun_out/gpu_all.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench/bench_pa.py --steps 10 --warmup 2 > gpurun_out/b_pa4.log 2>&1 || exit 1
tail -1 gpurun_out/b_pa4.log | cut -c1-200
timeout -k 10 300 python bench.py > gpurun_out/b_mf_final.log 2>&1 || exit 1
tail -1 gpurun_out/b_mf_final.log | cut -c1-200
timeout -k 10 300 python bench/bench_topk.py > gpurun_out/b_topk.log 2>&1 || exit 1
tail -1 gpurun_out/b_topk.log | cut -c1-300
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 1
tail -2 gpurun_out/smoke.log
echo ALLDONE
