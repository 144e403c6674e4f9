#!/bin/bash
# Round 5: geometric segment growth (2 = doubling) vs 3 / 4 -- LEMP and MF + top-K, alternating; top-K tests at 4.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5y
mkdir -p $O
echo skip-tests

for r in 1 2; do
  for g in 2 3 4; do
    FPS_TOPK_GROWTH=$g timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_g${g}_$r.log 2>&1 || { tail -20 $O/topk_g${g}_$r.log; exit 1; }
    echo "topk growth=$g $r $(tail -1 $O/topk_g${g}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
    FPS_TOPK_GROWTH=$g timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_g${g}_$r.log 2>&1 || { tail -20 $O/mftopk_g${g}_$r.log; exit 1; }
    echo "mftopk growth=$g $r $(tail -1 $O/mftopk_g${g}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
echo ALLDONE
