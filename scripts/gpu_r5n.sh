#!/bin/bash
# Round 5: wave-per-row fresh top-k selection (the scan's seed segment) -- numerics vs the block merge, top-K tests,
# LEMP + MF/top-K benches; the capped-grid partition test.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "topk_select or capped_grid" -x -v --timeout 300 --timeout-method thread > $O/tests_k.log 2>&1 || { tail -40 $O/tests_k.log; exit 1; }
grep -cE "PASSED" $O/tests_k.log
timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_topk.log 2>&1 || { tail -40 $O/tests_topk.log; exit 1; }
tail -1 $O/tests_topk.log
for i in 1 2; do
  timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_$i.log 2>&1 || { tail -20 $O/topk_$i.log; exit 1; }
  tail -1 $O/topk_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("topk", round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])'
done
for i in 1 2; do
  timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_$i.log 2>&1 || { tail -20 $O/mftopk_$i.log; exit 1; }
  tail -1 $O/mftopk_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("mftopk", round(d["ms_per_step"],3), "%.4e" % d["value"])'
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk -- python bench/bench_topk.py --steps 20 --warmup 3 > $O/prof_topk.log 2>&1 || { tail -20 $O/prof_topk.log; exit 1; }
echo ALLDONE
