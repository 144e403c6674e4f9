#!/bin/bash
# Round 4: virtual-world (RCCL-semantics) GPU tests only.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4c
timeout -k 10 600 python -u -m pytest tests/test_vworld_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r4c/vworld.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/r4c/vworld.log | tail -40
exit $rc
