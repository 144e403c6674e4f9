#!/bin/bash
# GPU: full gpu tests; prefetch vs not; profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 700 python -m pytest tests -q -m gpu > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> gpurun_out/gpu_tests.log
tail -6 gpurun_out/gpu_tests.log
case $rc in 0|1) ;; *) echo "stopping after test rc=$rc"; exit $rc;; esac
timeout -k 10 300 python bench.py > gpurun_out/b_prefetch.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --exchange rotate > gpurun_out/b_prefetch_rot.log 2>&1 || exit 1
for f in b_prefetch b_prefetch_rot; do tail -1 gpurun_out/$f.log | cut -c1-200; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/prefetch -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_prefetch.log 2>&1 || exit 1
echo ALLDONE
