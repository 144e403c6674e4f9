#!/bin/bash
# Round 6 (session 2): PA at N = 8 with the emulator's wait-timing events moved to a pass of their own (the timed
# loop runs without them, as a real RCCL job has none).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6aj
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_emulated_hot_owner.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"), "host", d.get("host_enqueue_ms_per_step"))')"
}
for r in 1 2; do
  run pa8_hash_$r python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
  run pa4_hash_$r python bench/bench_pa.py --emulate-world 4 --steps 80 --warmup 5 --partition hash
  run pa2_hash_$r python bench/bench_pa.py --emulate-world 2 --steps 80 --warmup 5 --partition hash
done
run pa8_range python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition range
run pa8_hash_host python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash --host-profile $O/pa8_host.txt
echo ALLDONE
