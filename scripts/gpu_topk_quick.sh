#!/bin/bash
# top-K GPU tests + both top-K benches + an MF+top-K kernel profile (one MI355X)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_topk_fast.py tests/test_topk_tensor_gpu.py tests/test_topk_tensor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mftopk_tests.log 2>&1 || { tail -30 gpurun_out/mftopk_tests.log; exit 1; }
tail -1 gpurun_out/mftopk_tests.log
timeout -k 10 300 python -u bench/bench_mf_topk.py --batch 4096 --steps 20 --warmup 3 > gpurun_out/mftopk_b4096.json && cat gpurun_out/mftopk_b4096.json
timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/topk.json && cat gpurun_out/topk.json
rm -rf gpurun_out/mftopk_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mftopk_prof -- python -u bench/bench_mf_topk.py --batch 4096 --steps 10 --warmup 2 > gpurun_out/mftopk_prof.log 2>&1
