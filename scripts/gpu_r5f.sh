#!/bin/bash
# Round 5: exact user rows (hogwild tests, bench + emulated N = 8 per user-update mode) and the secondary PS paths
# (PA pipelined, SGNS bf16 wire) at N = 1 / 2 / 4 / 8 under the rank-symmetric emulation, 50 and 100 GB/s links.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hogwild_gpu.py -x -v --timeout 500 --timeout-method thread > $O/hogwild.log 2>&1 || { tail -40 $O/hogwild.log; exit 1; }
grep -E "PASS|FAIL" $O/hogwild.log
timeout -k 10 300 python -c "
import sys, json; sys.path.insert(0, 'bench')
from probe_hogwild import lost_updates
for uu in ('store', 'atomic'):
    print(json.dumps(lost_updates(156_250, 125_000, 51.2, 1, user_update=uu, world=8)))
    print(json.dumps(lost_updates(1_000_000, 100_000, 6.4, 1, user_update=uu)))
" > $O/hogwild_geo.jsonl 2>&1 || { tail -20 $O/hogwild_geo.jsonl; exit 1; }
cut -c1-330 $O/hogwild_geo.jsonl
for uu in atomic store; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --user-update $uu > $O/bench_$uu.log 2>&1 || { tail -20 $O/bench_$uu.log; exit 1; }
  tail -1 $O/bench_$uu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["user_update"], round(d["ms_per_step"],3), "%.4e" % d["value"], d["config"]["lost_user_update_fraction"], d["effective_updates_per_s"])'
  timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 10 --warmup 3 --user-update $uu > $O/emu8_$uu.log 2>&1 || { tail -20 $O/emu8_$uu.log; exit 1; }
  tail -1 $O/emu8_$uu.log | cut -c1-200
done
for G in 50 100; do
  for N in 2 4 8; do
    timeout -k 10 300 python bench/bench_pa.py --ps-path --emulate-world $N --link-gbps $G > $O/pa_${N}_$G.log 2>&1 || { tail -20 $O/pa_${N}_$G.log; exit 1; }
    timeout -k 10 300 python bench/bench_w2v.py --ps-path --emulate-world $N --link-gbps $G > $O/w2v_${N}_$G.log 2>&1 || { tail -20 $O/w2v_${N}_$G.log; exit 1; }
    for f in pa w2v; do echo "$f N=$N ${G}GB/s $(tail -1 $O/${f}_${N}_$G.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], d["exposed_wait_ms_per_step"], d["config"]["wire_dtype"], d["config"].get("staleness"))')"; done
  done
done
timeout -k 10 300 python bench/bench_pa.py --ps-path --no-fuse-local-push > $O/pa_1_delta.log 2>&1 || { tail -20 $O/pa_1_delta.log; exit 1; }
timeout -k 10 300 python bench/bench_w2v.py --ps-path --no-fuse-local-push > $O/w2v_1_delta.log 2>&1 || { tail -20 $O/w2v_1_delta.log; exit 1; }
for f in pa w2v; do echo "$f N=1 delta-buffer $(tail -1 $O/${f}_1_delta.log | cut -c1-140)"; done
echo ALLDONE
