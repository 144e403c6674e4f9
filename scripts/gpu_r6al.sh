#!/bin/bash
# Round 6 (session 2): workgroups of a link-timed fill (FPS_FILL_LINK_WGS 256 / 512 / 1024): PA / SGNS N = 8 PS paths
# and the MF rotation at N = 8 with 50 GB/s links.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6al
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k segment_fill -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
for w in 256 512 1024; do
  export FPS_FILL_LINK_WGS=$w
  run pa8_w$w python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
  run w2v8_w$w python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
  timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu8_w$w.jsonl 2>$O/emu8_w$w.err || { tail -20 $O/emu8_w$w.err; exit 1; }
  echo "emu8_w$w $(grep '^{' $O/emu8_w$w.jsonl | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["comm_wait_ms_per_step"],3))')"
done
echo ALLDONE
