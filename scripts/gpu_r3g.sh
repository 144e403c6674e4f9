#!/bin/bash
# Round 3: identity plans (MF PS path), static-plan dump fix, COORD prefetch, PA PS-path profile, user-phase A/B.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3g
timeout -k 10 600 python -u -m pytest tests/test_tensor_engine_gpu.py tests/test_topk_bf16_gpu.py tests/test_step_graph_gpu.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3g/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3g/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --force-ps-path --steps 10 > gpurun_out/r3g/mf_ps.log 2>&1 || { tail -20 gpurun_out/r3g/mf_ps.log; exit 1; }
tail -1 gpurun_out/r3g/mf_ps.log | cut -c1-200
for st in length coord lc:1.3; do
  timeout -k 10 300 python bench/bench_topk.py --strategy $st > gpurun_out/r3g/topk_$st.log 2>&1 || { tail -20 gpurun_out/r3g/topk_$st.log; exit 1; }
  tail -1 gpurun_out/r3g/topk_$st.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3g/prof_pa -- python bench/bench_pa.py --ps-path --steps 5 --warmup 1 > gpurun_out/r3g/prof_pa.log 2>&1 || { tail -20 gpurun_out/r3g/prof_pa.log; exit 1; }
tail -1 gpurun_out/r3g/prof_pa.log | cut -c1-200
timeout -k 10 300 python bench/bench_pa.py > gpurun_out/r3g/pa_direct.log 2>&1 || { tail -20 gpurun_out/r3g/pa_direct.log; exit 1; }
tail -1 gpurun_out/r3g/pa_direct.log | cut -c1-200
for P in 4 6 8; do
  timeout -k 10 300 python bench.py --user-phases $P > gpurun_out/r3g/p$P.log 2>&1 || { tail -20 gpurun_out/r3g/p$P.log; exit 1; }
  echo "P=$P $(tail -1 gpurun_out/r3g/p$P.log | cut -c1-160)"
done
echo ALLDONE
