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
for rep in 1 2; do
  FPS_KERNELS_SO=$GRAFT_REPO_ROOT/flink_parameter_server_1_amd/_lib/ab/libfps_kernels_a.so timeout -k 10 300 python bench/bench_w2v.py --mode standard > gpurun_out/r3h/w2v_a$rep.log 2>&1 || { tail -20 gpurun_out/r3h/w2v_a$rep.log; exit 1; }
  echo "A $(tail -1 gpurun_out/r3h/w2v_a$rep.log | cut -c1-150)"
  timeout -k 10 300 python bench/bench_w2v.py --mode standard > gpurun_out/r3h/w2v_b$rep.log 2>&1 || { tail -20 gpurun_out/r3h/w2v_b$rep.log; exit 1; }
  echo "B $(tail -1 gpurun_out/r3h/w2v_b$rep.log | cut -c1-150)"
done
timeout -k 10 300 python bench/probe_hogwild.py --phases 1,4 > gpurun_out/r3h/hogwild.log 2>&1 || { tail -20 gpurun_out/r3h/hogwild.log; exit 1; }
cat gpurun_out/r3h/hogwild.log
timeout -k 10 300 python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 4 > gpurun_out/r3h/hogwild_full.log 2>&1 || { tail -20 gpurun_out/r3h/hogwild_full.log; exit 1; }
cat gpurun_out/r3h/hogwild_full.log
echo ALLDONE
