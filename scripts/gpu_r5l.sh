#!/bin/bash
# Round 5: user_update "auto" (exact at N > 1) -- N-rank GPU tests, emulated N = 8 default vs store, N = 2 rehearsal.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_vworld_gpu.py tests/test_multigpu_nccl_gpu.py tests/test_multirank_gpu.py tests/test_mf_tiled_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; grep -E "FAILED|passed|failed" $O/tests.log | tail -2
for v in auto store; do
  timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 8 --warmup 2 --user-update $v > $O/emu8_$v.log 2>&1 || { tail -20 $O/emu8_$v.log; exit 1; }
  echo "emu8 $v $(tail -1 $O/emu8_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["user_update"], round(d["ms_per_step"],3), "%.4e" % d["updates_per_s_per_gpu"])')"
done
FPS_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 4194304 > $O/bench_n2.log 2>&1 || { tail -30 $O/bench_n2.log; exit 1; }
grep '^{' $O/bench_n2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("n2", d["config"]["user_update"], d["verify_ok"], d["config"]["lost_user_update_fraction"], "%.4e" % d["value"], d["effective_updates_per_s"])'
timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_topk.log 2>&1 || { tail -40 $O/tests_topk.log; exit 1; }
tail -1 $O/tests_topk.log
for i in 1 2; do
  timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_$i.log 2>&1 || { tail -20 $O/topk_$i.log; exit 1; }
  tail -1 $O/topk_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("topk", round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])'
done
timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk.log 2>&1 || { tail -20 $O/mftopk.log; exit 1; }
tail -1 $O/mftopk.log | cut -c1-300
echo ALLDONE
