#!/bin/bash
# Round 6: baseline headline on a fresh box + float-atomic row probe on cache-resident working sets.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6a
mkdir -p $O
for r in 1 2; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
  tail -1 $O/bench_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"],3), "%.4e" % d["value"], d["config"]["lost_user_update_fraction"])'
done
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --user-update atomic --no-hogwild-probe > $O/bench_atomic.log 2>&1 || { tail -20 $O/bench_atomic.log; exit 1; }
tail -1 $O/bench_atomic.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("atomic", round(d["ms_per_step"],3), "%.4e" % d["value"])'
FPS_PROBE_ROWS=1 timeout -k 10 300 python -u bench/probe_atomics.py > $O/probe_rows.jsonl 2>&1 || { tail -20 $O/probe_rows.jsonl; exit 1; }
cat $O/probe_rows.jsonl
echo ALLDONE
