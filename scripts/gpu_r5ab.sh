#!/bin/bash
# Round 5: a device-side delay before the staged partition (FPS_PART_DELAY_US) so the SGD launch it starts with
# fills the CUs first -- MF PS path and local headline, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ab
mkdir -p $O
for r in 1 2; do
  for d in 0 300 800; do
    FPS_PART_DELAY_US=$d timeout -k 10 300 python bench.py --steps 20 --warmup 3 --force-ps-path --no-hogwild-probe > $O/ps_d${d}_$r.log 2>&1 || { tail -20 $O/ps_d${d}_$r.log; exit 1; }
    echo "ps delay=$d $r $(tail -1 $O/ps_d${d}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
  for d in 0 300; do
    FPS_PART_DELAY_US=$d timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-hogwild-probe > $O/loc_d${d}_$r.log 2>&1 || { tail -20 $O/loc_d${d}_$r.log; exit 1; }
    echo "local delay=$d $r $(tail -1 $O/loc_d${d}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
echo ALLDONE
