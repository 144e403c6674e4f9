#!/bin/bash
# bf16 top-K: numerics + top-K GPU suites, both benches twice, kernel stats of each bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bq
timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_fast.py tests/test_topk_tensor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bq/tests.log 2>&1 || { tail -30 gpurun_out/bq/tests.log; exit 1; }
tail -1 gpurun_out/bq/tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/bq/topk.$rep.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench/bench_mf_topk.py > gpurun_out/bq/mftopk.$rep.json 2>/dev/null || exit 1
  echo "rep$rep topk $(cut -c1-140 gpurun_out/bq/topk.$rep.json | cut -d, -f2) mftopk $(cut -d, -f2,4 gpurun_out/bq/mftopk.$rep.json)"
done
rm -rf gpurun_out/bq/prof_*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bq/prof_mftopk -- python -u bench/bench_mf_topk.py --steps 10 --warmup 2 > gpurun_out/bq/prof_mftopk.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bq/prof_topk -- python -u bench/bench_topk.py > gpurun_out/bq/prof_topk.log 2>&1 || exit 1
echo ALLDONE
