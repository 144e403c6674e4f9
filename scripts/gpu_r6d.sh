#!/bin/bash
# Round 6: owner-stream PS pipeline -- virtual-world / multirank / tensor-engine GPU tests, then emulated PA / SGNS
# A/B (FPS_OWNER_STREAM=0 vs 1) at N = 2 / 4 / 8.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_multigpu_nccl_gpu.py tests/test_vworld_gpu.py tests/test_multirank_gpu.py tests/test_tensor_engine_gpu.py tests/test_tensor_contract_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for os in 0 1; do
  for n in 2 8; do
    FPS_OWNER_STREAM=$os timeout -k 10 120 python bench/bench_pa.py --emulate-world $n --steps 20 --warmup 3 --partition hash > $O/pa${n}_os$os.log 2>&1 || { tail -20 $O/pa${n}_os$os.log; exit 1; }
    echo "os=$os pa N=$n hash $(tail -1 $O/pa${n}_os$os.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", round(d["exposed_wait_ms_per_step"],3))')"
    FPS_OWNER_STREAM=$os timeout -k 10 120 python bench/bench_pa.py --emulate-world $n --steps 20 --warmup 3 --partition range > $O/par${n}_os$os.log 2>&1 || { tail -20 $O/par${n}_os$os.log; exit 1; }
    echo "os=$os pa N=$n range $(tail -1 $O/par${n}_os$os.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", round(d["exposed_wait_ms_per_step"],3))')"
    FPS_OWNER_STREAM=$os timeout -k 10 120 python bench/bench_w2v.py --emulate-world $n --steps 10 --warmup 3 > $O/w2v${n}_os$os.log 2>&1 || { tail -20 $O/w2v${n}_os$os.log; exit 1; }
    echo "os=$os w2v N=$n $(tail -1 $O/w2v${n}_os$os.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", round(d["exposed_wait_ms_per_step"],3))')"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --emulate-world 8 --steps 10 --warmup 3 --partition hash > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
echo ALLDONE
