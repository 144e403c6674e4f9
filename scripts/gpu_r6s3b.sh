#!/bin/bash
# Round 6 session 3: bf16 scorer with prefetch distance 2 (FPS_SB_PD=2: two register sets, stage st+2 issued at the
# start of stage st) vs 1 -- top-K tests under PD=2, same-box A/B alternating, then the MFMA-busy counter pass of PD=2.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3b
mkdir -p $O
FPS_SB_PD=2 timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_topk_seen_merge_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 2 1; do
    FPS_SB_PD=$v timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    echo "topk pd=$v $r $(tail -1 $O/topk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
    FPS_SB_PD=$v timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "mftopk pd=$v $r $(tail -1 $O/mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for v in 2 1; do
  rm -rf $O/mftopk_pd${v}
  FPS_SB_PD=$v timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/mftopk_pd${v} -- python bench/bench_mf_topk.py > $O/mftopk_pd${v}.log 2>&1 || { echo "FAIL pmc $v"; tail -5 $O/mftopk_pd${v}.log; exit 1; }
done
echo ALLDONE
