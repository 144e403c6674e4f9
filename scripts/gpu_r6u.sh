#!/bin/bash
# Round 6 (session 2): lanes-per-row segment fill -- tests, config #5 / PA / SGNS emulated N = 8 re-measured.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "segment_fill" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
run cap8 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8
run cap8_bf16 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8 --wire bf16
run pa8_hash python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash
run pa8_range python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition range
run w2v8 python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
run cap1 python bench/bench_capacity.py --steps 20 --warmup 3
echo ALLDONE
