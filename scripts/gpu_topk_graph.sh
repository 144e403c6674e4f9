#!/bin/bash
# hipGraph-captured top-K scan: numerics (graph == eager), the top-K GPU suites, and a same-box
# A/B (FPS_TOPK_GRAPH=0: eager launches) of both top-K benches, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tg
timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_fast.py tests/test_topk_tensor_gpu.py tests/test_topk_tensor.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tg/tests.log 2>&1 || { tail -40 gpurun_out/tg/tests.log; exit 1; }
tail -1 gpurun_out/tg/tests.log
for rep in 1 2; do
  for v in 0 1; do
    FPS_TOPK_GRAPH=$v timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/tg/topk_$v.$rep.json 2>gpurun_out/tg/topk_$v.$rep.err || { tail -20 gpurun_out/tg/topk_$v.$rep.err; exit 1; }
    FPS_TOPK_GRAPH=$v timeout -k 10 300 python -u bench/bench_mf_topk.py > gpurun_out/tg/mftopk_$v.$rep.json 2>gpurun_out/tg/mftopk_$v.$rep.err || { tail -20 gpurun_out/tg/mftopk_$v.$rep.err; exit 1; }
    echo "graph=$v rep$rep topk $(cut -d, -f2 gpurun_out/tg/topk_$v.$rep.json) mftopk $(cut -d, -f2 gpurun_out/tg/mftopk_$v.$rep.json)"
  done
done
