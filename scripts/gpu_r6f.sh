#!/bin/bash
# Round 6: interleaved schedule (PA default) vs owner stream vs plain; GPU multi-rank tests.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multigpu_nccl_gpu.py tests/test_vworld_gpu.py tests/test_multirank_gpu.py tests/test_tensor_engine_gpu.py tests/test_tensor_contract_gpu.py tests/test_pa_offline_tensor_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 120 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", d["exposed_wait_ms_per_step"] and round(d["exposed_wait_ms_per_step"],3))')"
}
for rep in 1 2; do
  run pa8_hash_interleave_$rep python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition hash
  FPS_OWNER_STREAM=1 run pa8_hash_owner_$rep python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition hash
done
for n in 2 4 8; do
  run pa${n}_hash python bench/bench_pa.py --emulate-world $n --steps 20 --warmup 3 --partition hash
  run pa${n}_range python bench/bench_pa.py --emulate-world $n --steps 20 --warmup 3 --partition range
  run w2v$n python bench/bench_w2v.py --emulate-world $n --steps 10 --warmup 3
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --emulate-world 8 --steps 10 --warmup 3 --partition hash > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
echo ALLDONE
