#!/bin/bash
# Round 6 (session 2): link model A/B, same box: serial (round 5: sleep then copy) vs timed fill (one kernel lasting
# the link time); MF rotation N = 4 / 8, SGNS / PA N = 8; kernel traces of the N = 8 rotation under both.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6aa
mkdir -p $O
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
for r in 1 2; do
  for m in serial timed; do
    timeout -k 10 300 env FPS_EMU_LINK=$m python bench/bench_emulate_world.py --ws 4,8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu_${m}_$r.jsonl 2>$O/emu_${m}_$r.err || { tail -20 $O/emu_${m}_$r.err; exit 1; }
    python - $O/emu_${m}_$r.jsonl $m <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print("emu", sys.argv[2], d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], round(d["comm_wait_ms_per_step"], 3))
PY
    run w2v8_${m}_$r env FPS_EMU_LINK=$m python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
    run pa8_${m}_$r env FPS_EMU_LINK=$m python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash
  done
done
for m in serial timed; do
  FPS_EMU_LINK=$m timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof8_$m -- python bench/bench_emulate_world.py --ws 8 --steps 4 --warmup 2 --link-gbps 50 > $O/prof8_$m.log 2>&1 || { tail -20 $O/prof8_$m.log; exit 1; }
done
echo ALLDONE
