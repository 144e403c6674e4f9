#!/bin/bash
# Round 5: adaptive items per scorer workgroup (short segments get >= 1024 workgroups) -- top-K tests, then a same-box
# A/B vs FPS_SB_MIN_WGS=0 (always 1024 items per workgroup), alternating; per-segment trace.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_topk_seen_merge_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1024 0; do
    FPS_SB_MIN_WGS=$v timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    echo "topk minwgs=$v $r $(tail -1 $O/topk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
    FPS_SB_MIN_WGS=$v timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "mftopk minwgs=$v $r $(tail -1 $O/mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk -- python bench/bench_topk.py --steps 20 --warmup 3 > $O/prof_topk.log 2>&1 || { tail -20 $O/prof_topk.log; exit 1; }
echo ALLDONE
