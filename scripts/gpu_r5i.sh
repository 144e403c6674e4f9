#!/bin/bash
# Round 5: deferred top-K results (query_async) -- GPU tests, LEMP bench sync vs pipelined A/B (same box, alternating).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log
for i in 1 2; do
  for v in sync async; do
    F=""; [ $v = sync ] && F="--sync"
    timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 $F > $O/topk_${v}_$i.log 2>&1 || { tail -20 $O/topk_${v}_$i.log; exit 1; }
    tail -1 $O/topk_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("topk", sys.argv[1], round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])' $v
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk -- python bench/bench_topk.py --steps 20 --warmup 3 > $O/prof_topk.log 2>&1 || { tail -20 $O/prof_topk.log; exit 1; }
echo ALLDONE
