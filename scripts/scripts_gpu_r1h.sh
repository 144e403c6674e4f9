#!/bin/bash
# GPU pass: gpu tests; MF rotate-at-N=1 overhead; item-table size effect on the flat kernel (block sizes seen at N=2..8).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 700 python -m pytest tests -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
tail -4 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py --exchange rotate > gpurun_out/b_rot1.log 2>&1 || exit 1
for it in 500000 125000 62500; do
  timeout -k 10 300 python bench.py --items $it --steps 20 > gpurun_out/b_items$it.log 2>&1 || exit 1
done
for f in b_rot1 b_items500000 b_items125000 b_items62500; do tail -1 gpurun_out/$f.log | cut -c1-200; done
timeout -k 10 300 python bench/bench_pa.py --steps 10 --warmup 2 > gpurun_out/b_pa.log 2>&1 || exit 1
tail -1 gpurun_out/b_pa.log | cut -c1-300
echo ALLDONE
