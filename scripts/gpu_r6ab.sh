#!/bin/bash
# Round 6 (session 2): why the emulated N = 8 rotation step is ~7 ms under rocprofv3 but 8.7-10 ms in bench runs:
# step count, process order (the serial model's sleep is calibrated in clock cycles once per process), host time.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ab
mkdir -p $O
emu() {  # name, env..., -- args
  local n=$1; shift
  timeout -k 10 300 env "$@" > $O/$n.jsonl 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python - $O/$n.jsonl $n <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print("emu", sys.argv[2], d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], round(d["comm_wait_ms_per_step"], 3))
PY
}
for m in serial timed; do
  emu ${m}_248 FPS_EMU_LINK=$m python bench/bench_emulate_world.py --ws 2,4,8 --steps 20 --warmup 5 --link-gbps 50
  emu ${m}_8 FPS_EMU_LINK=$m python bench/bench_emulate_world.py --ws 8 --steps 20 --warmup 5 --link-gbps 50
  emu ${m}_8_s4 FPS_EMU_LINK=$m python bench/bench_emulate_world.py --ws 8 --steps 4 --warmup 2 --link-gbps 50
done
emu nolink_8 python bench/bench_emulate_world.py --ws 8 --steps 20 --warmup 5
echo ALLDONE
