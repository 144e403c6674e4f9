#!/bin/bash
# Round 5: online MF + top-K with its index pinned to doubling segments; LEMP; MF PS-path op table.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5aa
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_topk_tensor_gpu.py tests/test_vworld_gpu.py -k "topk" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_$r.log 2>&1 || { tail -20 $O/mftopk_$r.log; exit 1; }
  echo "mftopk $r $(tail -1 $O/mftopk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
for r in 1 2; do
  timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_$r.log 2>&1 || { tail -20 $O/topk_$r.log; exit 1; }
  echo "topk $r $(tail -1 $O/topk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
done
timeout -k 10 400 python bench/diag_ps_ops.py > $O/ps_ops.txt 2>&1 || { tail -20 $O/ps_ops.txt; exit 1; }
echo ALLDONE
