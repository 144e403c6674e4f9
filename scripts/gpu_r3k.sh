#!/bin/bash
# Round 3: secondary benches on the current tree (top-K strategies with focus-grouped queries, SGNS standard
# in place and through the PS path, MF PS path, MF + top-K serving).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3k
timeout -k 10 600 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3k/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3k/tests.log
[ $rc -eq 0 ] || exit 1
for st in length coord lc:1.3 li:5:2.5; do
  timeout -k 10 300 python bench/bench_topk.py --strategy $st > gpurun_out/r3k/topk_$st.log 2>&1 || { tail -20 gpurun_out/r3k/topk_$st.log; exit 1; }
  echo "topk $st $(tail -1 gpurun_out/r3k/topk_$st.log | cut -c1-120)"
done
timeout -k 10 300 python bench/bench_w2v.py --mode standard > gpurun_out/r3k/w2v_std.log 2>&1 || { tail -20 gpurun_out/r3k/w2v_std.log; exit 1; }
echo "w2v std $(tail -1 gpurun_out/r3k/w2v_std.log | cut -c1-140)"
timeout -k 10 300 python bench/bench_w2v.py --mode standard --ps-path > gpurun_out/r3k/w2v_std_ps.log 2>&1 || { tail -20 gpurun_out/r3k/w2v_std_ps.log; exit 1; }
echo "w2v std ps $(tail -1 gpurun_out/r3k/w2v_std_ps.log | cut -c1-140)"
timeout -k 10 300 python bench.py --force-ps-path --steps 10 > gpurun_out/r3k/mf_ps.log 2>&1 || { tail -20 gpurun_out/r3k/mf_ps.log; exit 1; }
echo "mf ps $(tail -1 gpurun_out/r3k/mf_ps.log | cut -c1-140)"
timeout -k 10 300 python bench/bench_mf_topk.py > gpurun_out/r3k/mf_topk.log 2>&1 || { tail -20 gpurun_out/r3k/mf_topk.log; exit 1; }
echo "mf topk $(tail -1 gpurun_out/r3k/mf_topk.log | cut -c1-160)"
echo ALLDONE
