#!/bin/bash
# GPU pass: gpu tests, headline bench (32M batch) local vs rotate-at-N=1, capacity, rotation profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 700 python -m pytest tests -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
tail -8 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py > gpurun_out/b_default.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --exchange rotate > gpurun_out/b_rot1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --batch 4194304 > gpurun_out/b_4m.log 2>&1 || exit 1
timeout -k 10 400 python bench/bench_capacity.py --steps 20 --warmup 3 > gpurun_out/b_cap.log 2>&1 || exit 1
for f in b_default b_rot1 b_4m b_cap; do tail -1 gpurun_out/$f.log | cut -c1-330; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/rot1 -- python bench.py --exchange rotate --steps 5 --warmup 1 > gpurun_out/prof_rot1.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/cap2 -- python bench/bench_capacity.py --steps 5 --warmup 1 > gpurun_out/prof_cap2.log 2>&1 || exit 1
echo ALLDONE
