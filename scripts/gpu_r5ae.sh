#!/bin/bash
# Round 5: the partition's side stream at high priority (FPS_PART_PRIORITY=-1) vs normal -- headline, PS path,
# emulated N = 8 (Hogwild), alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ae
mkdir -p $O
for r in 1 2; do
  for p in 0 -1; do
    FPS_PART_PRIORITY=$p timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-hogwild-probe > $O/loc_p${p}_$r.log 2>&1 || { tail -20 $O/loc_p${p}_$r.log; exit 1; }
    echo "local prio=$p $r $(tail -1 $O/loc_p${p}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
    FPS_PART_PRIORITY=$p timeout -k 10 300 python bench.py --steps 20 --warmup 3 --force-ps-path --no-hogwild-probe > $O/ps_p${p}_$r.log 2>&1 || { tail -20 $O/ps_p${p}_$r.log; exit 1; }
    echo "ps prio=$p $r $(tail -1 $O/ps_p${p}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
echo ALLDONE
