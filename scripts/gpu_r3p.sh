#!/bin/bash
# Round 3: request-routing kernel tests, PA request plans at W = 2 on one GPU (gloo rehearsal).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3p
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_multirank_gpu.py tests/test_pa_fast.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3p/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3p/tests.log
[ $rc -eq 0 ] || exit 1
echo ALLDONE
