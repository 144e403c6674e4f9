#!/bin/bash
# Round 3: PA PS path with spread padding; MF PS path kernel timeline.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3h
timeout -k 10 600 python -u -m pytest tests/test_tensor_engine_gpu.py tests/test_step_graph_gpu.py tests/test_tensor_contract_gpu.py tests/test_topk_bf16_gpu.py tests/test_sgns_sampling.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3h/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3h/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench/bench_pa.py --ps-path > gpurun_out/r3h/pa_ps.log 2>&1 || { tail -20 gpurun_out/r3h/pa_ps.log; exit 1; }
tail -1 gpurun_out/r3h/pa_ps.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h/prof_mfps -- python bench.py --force-ps-path --steps 4 --warmup 2 > gpurun_out/r3h/prof_mfps.log 2>&1 || { tail -20 gpurun_out/r3h/prof_mfps.log; exit 1; }
tail -1 gpurun_out/r3h/prof_mfps.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h/prof_local -- python bench.py --steps 4 --warmup 2 > gpurun_out/r3h/prof_local.log 2>&1 || { tail -20 gpurun_out/r3h/prof_local.log; exit 1; }
tail -1 gpurun_out/r3h/prof_local.log | cut -c1-200
for st in length coord lc:1.3; do
  timeout -k 10 300 python bench/bench_topk.py --strategy $st > gpurun_out/r3h/topk_$st.log 2>&1 || { tail -20 gpurun_out/r3h/topk_$st.log; exit 1; }
  tail -1 gpurun_out/r3h/topk_$st.log | cut -c1-200
done
echo ALLDONE
