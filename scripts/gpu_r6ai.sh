#!/bin/bash
# Round 6 (session 2): PS-path GPU time -- dynamic plans keep fresh dedup outputs (no per-plan clones); PA at N = 8
# with staleness 1 (default) and 2 and with the bf16 wire; GPU tests of the PS paths.  (r6ai: + segment fill 8 rows per lane per trip)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ai
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_emulated_hot_owner.py tests/test_kernels_gpu.py tests/test_pa_offline_tensor_gpu.py tests/test_tensor_engine_gpu.py tests/test_static_plan_gpu.py tests/test_multigpu_nccl_gpu.py tests/test_vworld_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"), "host", d.get("host_enqueue_ms_per_step"))')"
}
run pa8_hash_1 python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
run pa8_hash_2 python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
run pa8_range python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition range
run pa1_ps python bench/bench_pa.py --steps 80 --warmup 5 --partition hash --ps-path
run w2v8 python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
run cap8_bf16 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8 --wire bf16
timeout -k 10 400 python bench/bench_emulate_world.py --ws 8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu8.jsonl 2>$O/emu8.err || { tail -20 $O/emu8.err; exit 1; }
tail -1 $O/emu8.jsonl | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 5 --partition hash > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
echo ALLDONE
