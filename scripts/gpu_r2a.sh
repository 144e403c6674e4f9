#!/bin/bash
# Round 2: tensor engine GPU tests + the existing GPU suite subset touched by the TensorPS changes.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2a
timeout -k 10 600 python -u -m pytest tests/test_tensor_engine_gpu.py tests/test_kernels_gpu.py tests/test_pa_fast.py tests/test_emb_pairs.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2a/tests.log 2>&1; rc=$?
tail -30 gpurun_out/r2a/tests.log
exit $rc
