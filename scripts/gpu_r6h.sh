#!/bin/bash
# Round 6: scalar gather / apply kernels (D = 1): kernel tests, PA emulated N = 2/4/8, kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_touch_sentinel.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 120 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", d["exposed_wait_ms_per_step"] and round(d["exposed_wait_ms_per_step"],3), "acc", round(d["train_batch_accuracy"],3))')"
}
run pa1_ps python bench/bench_pa.py --ps-path --steps 20 --warmup 3 --partition hash
run pa1_ps_nofuse python bench/bench_pa.py --ps-path --no-fuse-local-push --steps 20 --warmup 3 --partition hash
for n in 2 4 8; do
  run pa${n}_hash python bench/bench_pa.py --emulate-world $n --steps 20 --warmup 3 --partition hash
  run pa${n}_range python bench/bench_pa.py --emulate-world $n --steps 20 --warmup 3 --partition range
done
run pa8_hash_z0 python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition hash --zipf 0
run pa8_range_z0 python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition range --zipf 0
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --emulate-world 8 --steps 10 --warmup 3 --partition hash > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
echo ALLDONE
