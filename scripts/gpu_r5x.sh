#!/bin/bash
# Round 5: user phases per step (4 = auto at 10M users) vs 6 / 8 -- headline A/B, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5x
mkdir -p $O
for r in 1 2; do
  for p in 0 6 8; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --user-phases $p > $O/ab_p${p}_$r.log 2>&1 || { tail -20 $O/ab_p${p}_$r.log; exit 1; }
    echo "phases $p $r $(tail -1 $O/ab_p${p}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(c["user_phases"], round(d["ms_per_step"],3), "%.4e" % d["value"], c["lost_user_update_fraction"], "%.4e" % d["effective_updates_per_s"])')"
  done
done
for r in 1 2; do
  for m in 256 384 512 1024; do
    FPS_SB_MIN_WGS=$m timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_m${m}_$r.log 2>&1 || { tail -20 $O/topk_m${m}_$r.log; exit 1; }
    echo "topk minwgs=$m $r $(tail -1 $O/topk_m${m}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
    FPS_SB_MIN_WGS=$m timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_m${m}_$r.log 2>&1 || { tail -20 $O/mftopk_m${m}_$r.log; exit 1; }
    echo "mftopk minwgs=$m $r $(tail -1 $O/mftopk_m${m}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
echo ALLDONE
