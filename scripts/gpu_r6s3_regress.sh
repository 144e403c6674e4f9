#!/bin/bash
# Round 6 session 3: is the headline's slide since round 3 (driver 1.069e10 -> 1.016e10) code or box?  The
# round-3 and round-5 driver commits (git worktrees under ab/, built in-tree) against HEAD, same box, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6s3reg
mkdir -p $O
for r in 1 2 3; do
  for v in r03 r05 head; do
    if [ $v = head ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/ab/$v; fi
    (cd $d && timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/${v}_$r.log 2>&1) || { tail -20 $O/${v}_$r.log; exit 1; }
    echo "$v $r $(grep '^{' $O/${v}_$r.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
echo ALLDONE
