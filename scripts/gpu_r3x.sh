#!/bin/bash
# Round 3: GC disabled during hipGraph capture -- the order that aborted before (engine tests first, leaving
# pinned host tensors / events as garbage, then the graph-capture tests in the same process).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3x
timeout -k 10 600 python -u -m pytest tests/test_tensor_engine_gpu.py tests/test_step_graph_gpu.py tests/test_sgns_sampling.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3x/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3x/tests.log
[ $rc -eq 0 ] || exit 1
echo ALLDONE
