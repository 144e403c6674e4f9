#!/bin/bash
# Round 6 (session 2): does the emulated N = 8 rotation depend on the N run before it in the process (the serial
# model's sleep is calibrated in clock cycles once per process)?  serial vs timed, --ws 2,4,8 vs --ws 8.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ab
mkdir -p $O
for m in serial timed; do
  for ws in 2,4,8 8; do
    timeout -k 10 300 env FPS_EMU_LINK=$m python bench/bench_emulate_world.py --ws $ws --steps 20 --warmup 5 --link-gbps 50 > $O/emu_${m}_${ws}.jsonl 2>$O/emu_${m}_${ws}.err || { tail -20 $O/emu_${m}_${ws}.err; exit 1; }
    python - $O/emu_${m}_${ws}.jsonl $m $ws <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print("emu", sys.argv[2], "ws=" + sys.argv[3], d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], round(d["comm_wait_ms_per_step"], 3))
PY
  done
done
echo ALLDONE
