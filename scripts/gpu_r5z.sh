#!/bin/bash
# Round 5: adaptive segment growth + scorer floor 512 -- top-K GPU tests, LEMP and MF + top-K benches, kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_topk_seen_merge_gpu.py tests/test_kernels_gpu.py -k "topk or score or lemp or Lemp" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_$r.log 2>&1 || { tail -20 $O/topk_$r.log; exit 1; }
  echo "topk $r $(tail -1 $O/topk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
  timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_$r.log 2>&1 || { tail -20 $O/mftopk_$r.log; exit 1; }
  echo "mftopk $r $(tail -1 $O/mftopk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk -- python bench/bench_topk.py --steps 20 --warmup 3 > $O/prof_topk.log 2>&1 || { tail -20 $O/prof_topk.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py > $O/prof_mftopk.log 2>&1 || { tail -20 $O/prof_mftopk.log; exit 1; }
echo ALLDONE
