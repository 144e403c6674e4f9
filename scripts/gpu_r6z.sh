#!/bin/bash
# Round 6 (session 2): link fills capped at 256 workgroups; N = 8 kernel trace of the rotation with links.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6z
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench/bench_emulate_world.py --ws 4,8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu_links_$r.jsonl 2>$O/emu_links_$r.err || { tail -20 $O/emu_links_$r.err; exit 1; }
  python - $O/emu_links_$r.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print("emu_links", d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], round(d["comm_wait_ms_per_step"], 3))
PY
done
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
run pa8_hash python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash
run w2v8 python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
run cap8_bf16 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8 --wire bf16
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof8 -- python bench/bench_emulate_world.py --ws 8 --steps 4 --warmup 2 --link-gbps 50 > $O/prof8.log 2>&1 || { tail -20 $O/prof8.log; exit 1; }
echo ALLDONE
