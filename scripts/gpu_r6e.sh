#!/bin/bash
# Round 6: PA / SGNS emulated N > 1 after the one-kernel link fill: owner stream A/B, dedup A/B, timeline profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e
mkdir -p $O
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 120 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", d["exposed_wait_ms_per_step"] and round(d["exposed_wait_ms_per_step"],3))')"
}
for os in 0 1; do
  for dd in auto on; do
    FPS_OWNER_STREAM=$os run pa8_hash_os${os}_dd$dd python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition hash --dedup $dd
  done
  FPS_OWNER_STREAM=$os run pa2_hash_os$os python bench/bench_pa.py --emulate-world 2 --steps 20 --warmup 3 --partition hash
  FPS_OWNER_STREAM=$os run pa8_range_os$os python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition range
  FPS_OWNER_STREAM=$os run w2v8_os$os python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
done
run pa1_ps_hash python bench/bench_pa.py --ps-path --steps 20 --warmup 3 --partition hash
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --emulate-world 8 --steps 10 --warmup 3 --partition hash > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2v8 -- python bench/bench_w2v.py --emulate-world 8 --steps 6 --warmup 2 > $O/prof_w2v8.log 2>&1 || { tail -20 $O/prof_w2v8.log; exit 1; }
echo ALLDONE
