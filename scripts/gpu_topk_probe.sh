#!/bin/bash
# top-K scorer probe + GPU top-K tests + the two top-K benches (one MI355X)
set -e
mkdir -p gpurun_out
timeout -k 10 200 python scripts/probe_score.py > gpurun_out/probe_score.json
timeout -k 10 400 python -u -m pytest tests/test_topk_fast.py tests/test_topk_tensor_gpu.py tests/test_topk_tensor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mftopk_tests.log 2>&1 || { tail -30 gpurun_out/mftopk_tests.log; exit 1; }
tail -2 gpurun_out/mftopk_tests.log
timeout -k 10 300 python -u bench/bench_mf_topk.py --batch 4096 --steps 20 --warmup 3 > gpurun_out/mftopk_b4096.json && cat gpurun_out/mftopk_b4096.json
FPS_TOPK_SYNC_SCAN=1 timeout -k 10 300 python -u bench/bench_mf_topk.py --batch 4096 --steps 20 --warmup 3 > gpurun_out/mftopk_b4096_sync.json && cat gpurun_out/mftopk_b4096_sync.json
timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/topk.json && cat gpurun_out/topk.json
FPS_TOPK_SYNC_SCAN=1 timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/topk_sync.json && cat gpurun_out/topk_sync.json
