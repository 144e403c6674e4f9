#!/bin/bash
# Round 3 (re-entry): GPU tests of the latest tree (incl. hipGraph step replay), engine plumbing eager vs
# graph, PS-path benches, LEMP strategies, headline bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3f
timeout -k 10 900 python -u -m pytest tests/test_step_graph_gpu.py tests/test_sgns_sampling.py tests/test_tensor_engine_gpu.py tests/test_tensor_contract_gpu.py \
  tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_pa_offline_tensor_gpu.py tests/test_mf_tiled_gpu.py \
  tests/test_multirank_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3f/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3f/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench/bench_engine.py --batches 1,64,4096,262144 > gpurun_out/r3f/engine.log 2>&1 || { tail -20 gpurun_out/r3f/engine.log; exit 1; }
tail -1 gpurun_out/r3f/engine.log | cut -c1-900
timeout -k 10 300 python bench/bench_engine.py --graph --batches 1,64,4096,262144 > gpurun_out/r3f/engine_graph.log 2>&1 || { tail -20 gpurun_out/r3f/engine_graph.log; exit 1; }
tail -1 gpurun_out/r3f/engine_graph.log | cut -c1-900
timeout -k 10 300 python bench/bench_pa.py --ps-path > gpurun_out/r3f/pa_ps.log 2>&1 || { tail -20 gpurun_out/r3f/pa_ps.log; exit 1; }
tail -1 gpurun_out/r3f/pa_ps.log | cut -c1-300
timeout -k 10 300 python bench.py --force-ps-path --steps 10 > gpurun_out/r3f/mf_ps.log 2>&1 || { tail -20 gpurun_out/r3f/mf_ps.log; exit 1; }
tail -1 gpurun_out/r3f/mf_ps.log | cut -c1-200
for st in length coord lc:1.3 li:5:2.5; do
  timeout -k 10 300 python bench/bench_topk.py --strategy $st > gpurun_out/r3f/topk_$st.log 2>&1 || { tail -20 gpurun_out/r3f/topk_$st.log; exit 1; }
  tail -1 gpurun_out/r3f/topk_$st.log | cut -c1-420
done
timeout -k 10 300 python bench.py > gpurun_out/r3f/bench_n1.log 2>&1 || { tail -20 gpurun_out/r3f/bench_n1.log; exit 1; }
tail -1 gpurun_out/r3f/bench_n1.log | cut -c1-200
timeout -k 10 300 python bench/bench_w2v.py --mode standard > gpurun_out/r3f/w2v_sorted.log 2>&1 || { tail -20 gpurun_out/r3f/w2v_sorted.log; exit 1; }
tail -1 gpurun_out/r3f/w2v_sorted.log | cut -c1-300
FPS_SGNS_METHOD=atomic timeout -k 10 300 python bench/bench_w2v.py --mode standard > gpurun_out/r3f/w2v_atomic.log 2>&1 || { tail -20 gpurun_out/r3f/w2v_atomic.log; exit 1; }
tail -1 gpurun_out/r3f/w2v_atomic.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f/prof_w2v -- python bench/bench_w2v.py --mode standard --steps 5 --warmup 1 > gpurun_out/r3f/prof_w2v.log 2>&1 || { tail -20 gpurun_out/r3f/prof_w2v.log; exit 1; }
echo ALLDONE
