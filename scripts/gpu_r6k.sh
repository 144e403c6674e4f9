#!/bin/bash
# Round 6: emulated MF rotation scaling (Hogwild default at every N, + exact mode), capacity N = 8 bf16 wire,
# SGNS interleaved A/B, PA final table; headline kernel profile of the timed loop only.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 400 python bench/bench_emulate_world.py --ws 1,2,4,8 --steps 20 --warmup 5 > $O/emu.jsonl 2>$O/emu.err || { tail -20 $O/emu.err; exit 1; }
timeout -k 10 300 python bench/bench_emulate_world.py --ws 2,8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu_links.jsonl 2>$O/emu_links.err || { tail -20 $O/emu_links.err; exit 1; }
timeout -k 10 300 python bench/bench_emulate_world.py --ws 2,8 --steps 10 --warmup 3 --user-update atomic > $O/emu_atomic.jsonl 2>$O/emu_atomic.err || { tail -20 $O/emu_atomic.err; exit 1; }
python - <<'PY'
import json
for f in ("emu", "emu_links", "emu_atomic"):
    for l in open(f"gpurun_out/r6k/{f}.jsonl"):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], d["user_update"], d["comm_wait_ms_per_step"])
PY
runc() {
  local n=$1; shift
  timeout -k 10 300 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["value"], "pairs/s %.3e" % d["pairs_per_s"], "wait", d.get("exposed_wait_ms_per_step"), "hbm", round(d["peak_hbm_gib_rank0"],1), "rank", d.get("emulated_rank"), d["config"].get("owner_stream"), d["config"].get("interleaved"))')"
}
runc cap8_bf16 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8 --wire bf16
FPS_OWNER_STREAM=0 runc cap8_bf16_noowner python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8 --wire bf16
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 150 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", d["exposed_wait_ms_per_step"] and round(d["exposed_wait_ms_per_step"],3))')"
}
FPS_OWNER_STREAM=0 run w2v8_interleave python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -- python bench.py --steps 20 --warmup 5 --no-hogwild-probe --exact-steps 0 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log | cut -c1-200
echo ALLDONE
