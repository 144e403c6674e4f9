#!/bin/bash
# Round 5: final top-K build -- top-K GPU tests, LEMP and MF + top-K end-to-end rates (3 runs each).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5an
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_topk_fast.py tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
for r in 1 2 3; do
  timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_$r.log 2>&1 || { tail -20 $O/topk_$r.log; exit 1; }
  echo "topk $r $(tail -1 $O/topk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_$r.log 2>&1 || { tail -20 $O/mftopk_$r.log; exit 1; }
  echo "mftopk $r $(tail -1 $O/mftopk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
timeout -k 10 300 python bench/diag_mf_topk_ops.py > gpurun_out/r5an/diag.txt 2>&1 || { tail -20 gpurun_out/r5an/diag.txt; exit 1; }
echo ALLDONE
