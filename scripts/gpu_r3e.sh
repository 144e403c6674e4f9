#!/bin/bash
# Round 3: static world-1 plans, MaskedPair outputs, LEMP COORD in the scorer -- GPU tests + benches.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3e
timeout -k 10 900 python -u -m pytest tests/test_tensor_engine_gpu.py tests/test_tensor_contract_gpu.py \
  tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_pa_offline_tensor_gpu.py tests/test_mf_tiled_gpu.py \
  tests/test_multirank_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3e/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3e/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench/bench_engine.py --batches 1,64,4096,262144 > gpurun_out/r3e/engine.log 2>&1 || { tail -20 gpurun_out/r3e/engine.log; exit 1; }
tail -1 gpurun_out/r3e/engine.log | cut -c1-700
timeout -k 10 300 python bench/bench_pa.py --ps-path > gpurun_out/r3e/pa_ps.log 2>&1 || { tail -20 gpurun_out/r3e/pa_ps.log; exit 1; }
tail -1 gpurun_out/r3e/pa_ps.log | cut -c1-160
timeout -k 10 300 python bench.py --force-ps-path --steps 10 > gpurun_out/r3e/mf_ps.log 2>&1 || { tail -20 gpurun_out/r3e/mf_ps.log; exit 1; }
tail -1 gpurun_out/r3e/mf_ps.log | cut -c1-160
for st in length coord lc:1.3 li:5:2.5; do
  timeout -k 10 300 python bench/bench_topk.py --strategy $st > gpurun_out/r3e/topk_$st.log 2>&1 || { tail -20 gpurun_out/r3e/topk_$st.log; exit 1; }
  tail -1 gpurun_out/r3e/topk_$st.log | cut -c1-420
done
timeout -k 10 300 python bench.py > gpurun_out/r3e/bench_n1.log 2>&1 || { tail -20 gpurun_out/r3e/bench_n1.log; exit 1; }
tail -1 gpurun_out/r3e/bench_n1.log | cut -c1-200
echo ALLDONE
