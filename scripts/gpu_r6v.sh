#!/bin/bash
# Round 6 (session 2): why the emulated N = 4 rotation step with 50 GB/s links is slower than N = 8 -- overlap on/off
# and a kernel trace of the N = 4 run.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6v
mkdir -p $O
for ov in auto off on; do
  timeout -k 10 300 python bench/bench_emulate_world.py --ws 2,4,8 --steps 20 --warmup 5 --link-gbps 50 --overlap $ov > $O/emu_$ov.jsonl 2>$O/emu_$ov.err || { tail -20 $O/emu_$ov.err; exit 1; }
  python - $O/emu_$ov.jsonl $ov <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(sys.argv[2], d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], round(d["comm_wait_ms_per_step"], 3))
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof4 -- python bench/bench_emulate_world.py --ws 4 --steps 6 --warmup 3 --link-gbps 50 > $O/prof4.log 2>&1 || { tail -20 $O/prof4.log; exit 1; }
echo ALLDONE
