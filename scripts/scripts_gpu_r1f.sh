#!/bin/bash
# GPU pass: full gpu test suite, headline + capacity + PA benches, capacity kernel profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 700 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
tail -5 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit $rc;; esac
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/b_default.log 2>&1 || exit 1
timeout -k 10 400 python bench/bench_capacity.py --steps 20 --warmup 3 > gpurun_out/b_cap.log 2>&1 || exit 1
timeout -k 10 400 python bench/bench_capacity.py --steps 20 --warmup 3 --optimizer adagrad > gpurun_out/b_cap_adagrad.log 2>&1 || exit 1
timeout -k 10 300 python bench/bench_pa.py --steps 10 --warmup 2 > gpurun_out/b_pa.log 2>&1 || exit 1
for f in b_default b_cap b_cap_adagrad b_pa; do tail -1 gpurun_out/$f.log | cut -c1-400; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/cap -- python bench/bench_capacity.py --steps 5 --warmup 1 > gpurun_out/prof_cap.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/pa -- python bench/bench_pa.py --steps 5 --warmup 1 > gpurun_out/prof_pa.log 2>&1 || exit 1
echo ALLDONE
