#!/bin/bash
# Round 5: scorer workgroup floor sweep (multiples of the 768 workgroup slots) -- LEMP and MF + top-K, alternating;
# MF + top-K kernel stats at the default.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5u
mkdir -p $O
for r in 1 2; do
  for v in 1024 1536 2304 3072; do
    FPS_SB_MIN_WGS=$v timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    echo "topk minwgs=$v $r $(tail -1 $O/topk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
    FPS_SB_MIN_WGS=$v timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "mftopk minwgs=$v $r $(tail -1 $O/mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py > $O/prof_mftopk.log 2>&1 || { tail -20 $O/prof_mftopk.log; exit 1; }
echo ALLDONE
