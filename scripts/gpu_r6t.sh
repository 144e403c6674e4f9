#!/bin/bash
# Round 6 (session 2): SGNS kernels read bf16 wire rows directly and write the bf16 push; tests + SGNS N = 1/2/4/8.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sgns_sampling.py -q -x -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
run w2v8 python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
run w2v8b python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
run w2v4 python bench/bench_w2v.py --emulate-world 4 --steps 10 --warmup 3
run w2v2 python bench/bench_w2v.py --emulate-world 2 --steps 10 --warmup 3
run w2v1_ps python bench/bench_w2v.py --steps 10 --warmup 3 --ps-path
run w2v1_ps_bf16 python bench/bench_w2v.py --steps 10 --warmup 3 --ps-path --wire bf16
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2v8 -- python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3 > $O/prof_w2v8.log 2>&1 || { tail -20 $O/prof_w2v8.log; exit 1; }
run pa8_hash python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash
run pa8_hash_b python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash
run pa1_ps python bench/bench_pa.py --ps-path --steps 40 --warmup 5 --partition hash
echo ALLDONE
