#!/bin/bash
# Round 3, first GPU pass: the new contract / hash-table tests, the tensor-engine GPU tests, the headline bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tensor_contract_gpu.py tests/test_tensor_engine_gpu.py \
  tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3a_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3a_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r3a_bench.log 2>&1 || { tail -20 gpurun_out/r3a_bench.log; exit 1; }
tail -1 gpurun_out/r3a_bench.log | cut -c1-250
