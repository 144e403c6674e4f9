#!/bin/bash
# Online MF + top-K serving bench (tensor engine) on one MI355X: GPU tests, A/B of the
# fused scorer tiles, the LEMP top-K bench, and a kernel profile.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_topk_fast.py tests/test_topk_tensor_gpu.py tests/test_topk_tensor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mftopk_tests.log 2>&1 || { tail -30 gpurun_out/mftopk_tests.log; exit 1; }
tail -2 gpurun_out/mftopk_tests.log
for b in 4096 16384; do
  timeout -k 10 300 python -u bench/bench_mf_topk.py --batch $b --steps 20 --warmup 3 > gpurun_out/mftopk_b$b.json
  cat gpurun_out/mftopk_b$b.json
done
FPS_TOPK_TILE64=1 timeout -k 10 300 python -u bench/bench_mf_topk.py --batch 4096 --steps 20 --warmup 3 > gpurun_out/mftopk_b4096_tile64.json
cat gpurun_out/mftopk_b4096_tile64.json
timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/topk.json && cat gpurun_out/topk.json
FPS_TOPK_TILE64=1 timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/topk_tile64.json && cat gpurun_out/topk_tile64.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mftopk_prof -- \
  python -u bench/bench_mf_topk.py --batch 4096 --steps 10 --warmup 2 > gpurun_out/mftopk_prof.log 2>&1
echo done
