#!/bin/bash
# Round 6 (session 2): is the PA PS path at N = 8 host-bound?  Host enqueue time vs wall time (no profiler), the same
# with the links removed, and a kernel trace for the GPU-busy time per step.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ad
mkdir -p $O
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"), "host", d.get("host_enqueue_ms_per_step"))')"
}
run pa8_hash_1 python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
run pa8_hash_2 python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
run pa8_hash_nolink python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash --link-gbps 1e6 --latency-us 0
run pa1_ps python bench/bench_pa.py --steps 80 --warmup 5 --partition hash --ps-path
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 5 --partition hash > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
echo ALLDONE
