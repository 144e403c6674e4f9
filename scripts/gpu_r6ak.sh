#!/bin/bash
# Round 6 (session 2): PA N = 8 host time per PS stage (wall-clock wrappers); count copy on the compute stream.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6ak
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_emulated_hot_owner.py tests/test_tensor_engine_gpu.py tests/test_multigpu_nccl_gpu.py tests/test_vworld_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash > $O/pa8_$r.log 2>&1 || { tail -20 $O/pa8_$r.log; exit 1; }
  tail -1 $O/pa8_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("pa8", round(d["ms_per_step"],3), "%.4g" % d["per_gpu_rate"], "wait", d.get("exposed_wait_ms_per_step"), "host", d.get("host_enqueue_ms_per_step"))'
done
timeout -k 10 200 python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash --host-breakdown > $O/pa8_bd.log 2>&1 || { tail -20 $O/pa8_bd.log; exit 1; }
grep "^host" $O/pa8_bd.log
tail -1 $O/pa8_bd.log | cut -c1-120
echo ALLDONE
