#!/bin/bash
# Round 6 (session 2): PS-path host time -- raw stream handles for kernel launches, the emulated exchange launched
# straight onto its link stream (no stream context / wait_stream), PA ids only when predictions are emitted.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6af
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_emulated_hot_owner.py tests/test_pa_fast.py tests/test_pa_offline_tensor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"), "host", d.get("host_enqueue_ms_per_step"))')"
}
run pa8_hash_1 python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
run pa8_hash_2 python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
run pa8_hash_nolink python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash --link-gbps 1e6 --latency-us 0
run pa1_ps python bench/bench_pa.py --steps 80 --warmup 5 --partition hash --ps-path
run w2v8 python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
run pa8_host python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash --host-profile $O/pa8_host.txt
echo ALLDONE
