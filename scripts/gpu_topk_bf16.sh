#!/bin/bash
# bf16 top-K scan: numerics tests, the top-K GPU suites, A/B of both top-K benches
# (FPS_TOPK_BF16=0: fp32 scorer) on one box, kernel stats of the MF + top-K bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bf16
timeout -k 10 300 python -u -m pytest tests/test_topk_bf16_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/bf16/tests_new.log 2>&1 || { tail -40 gpurun_out/bf16/tests_new.log; exit 1; }
tail -1 gpurun_out/bf16/tests_new.log
timeout -k 10 400 python -u -m pytest tests/test_topk_fast.py tests/test_topk_tensor_gpu.py tests/test_topk_tensor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bf16/tests_topk.log 2>&1 || { tail -30 gpurun_out/bf16/tests_topk.log; exit 1; }
tail -1 gpurun_out/bf16/tests_topk.log
for rep in 1 2; do
  for v in 0 1; do
    FPS_TOPK_BF16=$v timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/bf16/topk_$v.$rep.json 2>gpurun_out/bf16/topk_$v.$rep.err || { tail -20 gpurun_out/bf16/topk_$v.$rep.err; exit 1; }
    echo "topk bf16=$v $(cut -c1-160 gpurun_out/bf16/topk_$v.$rep.json)"
    FPS_TOPK_BF16=$v timeout -k 10 300 python -u bench/bench_mf_topk.py > gpurun_out/bf16/mftopk_$v.$rep.json 2>gpurun_out/bf16/mftopk_$v.$rep.err || { tail -20 gpurun_out/bf16/mftopk_$v.$rep.err; exit 1; }
    echo "mftopk bf16=$v $(cut -c1-200 gpurun_out/bf16/mftopk_$v.$rep.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bf16/prof_mftopk -- python -u bench/bench_mf_topk.py --steps 10 --warmup 2 > gpurun_out/bf16/prof_mftopk.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bf16/prof_topk -- python -u bench/bench_topk.py > gpurun_out/bf16/prof_topk.log 2>&1 || exit 1
echo ALLDONE
