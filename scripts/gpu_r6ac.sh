#!/bin/bash
# Round 6 (session 2): emulated MF rotation scaling with one fresh process per N; link model timed (default) vs serial.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ac
mkdir -p $O
show() {
  python - $1 $2 <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print(sys.argv[2], d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], round(d["comm_wait_ms_per_step"], 3))
PY
}
timeout -k 10 400 python bench/bench_emulate_world.py --ws 1,2,4,8 --steps 20 --warmup 5 > $O/emu.jsonl 2>$O/emu.err || { tail -20 $O/emu.err; exit 1; }
show $O/emu.jsonl emu
for r in 1 2; do
  timeout -k 10 400 python bench/bench_emulate_world.py --ws 2,4,8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu_links_$r.jsonl 2>$O/emu_links_$r.err || { tail -20 $O/emu_links_$r.err; exit 1; }
  show $O/emu_links_$r.jsonl emu_links_timed
  timeout -k 10 400 env FPS_EMU_LINK=serial python bench/bench_emulate_world.py --ws 2,4,8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu_links_serial_$r.jsonl 2>$O/emu_links_serial_$r.err || { tail -20 $O/emu_links_serial_$r.err; exit 1; }
  show $O/emu_links_serial_$r.jsonl emu_links_serial
done
echo ALLDONE
