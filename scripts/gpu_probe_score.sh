#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python scripts/probe_score.py > gpurun_out/probe_score2.json
timeout -k 10 400 python -u -m pytest tests/test_tensor_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/te_gpu.log 2>&1 || { tail -30 gpurun_out/te_gpu.log; exit 1; }
tail -1 gpurun_out/te_gpu.log
