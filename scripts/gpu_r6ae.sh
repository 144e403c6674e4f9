#!/bin/bash
# Round 6 (session 2): bf16 scorer with the query blocks' MFMA chains interleaved (FPS_SB_ILV=1, default) vs one chain
# at a time (0) -- top-K tests, same-box A/B alternating, then the MFMA-busy counter pass of both.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_topk_seen_merge_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    FPS_SB_ILV=$v timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    echo "topk ilv=$v $r $(tail -1 $O/topk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
    FPS_SB_ILV=$v timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "mftopk ilv=$v $r $(tail -1 $O/mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for v in 1 0; do
  rm -rf $O/mftopk_ilv${v}_1
  FPS_SB_ILV=$v timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/mftopk_ilv${v}_1 -- python bench/bench_mf_topk.py > $O/mftopk_ilv${v}_1.log 2>&1 || { echo "FAIL pmc $v"; tail -5 $O/mftopk_ilv${v}_1.log; exit 1; }
  rm -rf $O/topk_ilv${v}_1
  FPS_SB_ILV=$v timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/topk_ilv${v}_1 -- python bench/bench_topk.py --steps 6 --warmup 2 > $O/topk_ilv${v}_1.log 2>&1 || { echo "FAIL pmc topk $v"; tail -5 $O/topk_ilv${v}_1.log; exit 1; }
done
echo ALLDONE
