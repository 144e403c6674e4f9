#!/bin/bash
# Round 3: top-K scan without the per-segment count fill (B = tree) vs HEAD (A = _abtree, its own build), same box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3o
timeout -k 10 600 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_tensor_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3o/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3o/tests.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then R=_abtree; else R=.; fi
    timeout -k 10 300 python $R/bench/bench_topk.py > gpurun_out/r3o/topk_$v$rep.log 2>&1 || { tail -20 gpurun_out/r3o/topk_$v$rep.log; exit 1; }
    timeout -k 10 300 python $R/bench/bench_mf_topk.py > gpurun_out/r3o/mftopk_$v$rep.log 2>&1 || { tail -20 gpurun_out/r3o/mftopk_$v$rep.log; exit 1; }
    echo "$v$rep topk $(grep -o '"value": [0-9.e+]*' gpurun_out/r3o/topk_$v$rep.log) $(grep -o '"exact_vs_brute_force": [a-z]*' gpurun_out/r3o/topk_$v$rep.log) mftopk $(grep -o '"value": [0-9.e+]*' gpurun_out/r3o/mftopk_$v$rep.log)"
  done
done
for b in 131072 262144; do
  timeout -k 10 300 python bench/bench_topk.py --bucket $b > gpurun_out/r3o/topk_b$b.log 2>&1 || { tail -20 gpurun_out/r3o/topk_b$b.log; exit 1; }
  timeout -k 10 300 python bench/bench_mf_topk.py --bucket $b > gpurun_out/r3o/mftopk_b$b.log 2>&1 || { tail -20 gpurun_out/r3o/mftopk_b$b.log; exit 1; }
  echo "bucket $b topk $(grep -o '"value": [0-9.e+]*' gpurun_out/r3o/topk_b$b.log) mftopk $(grep -o '"value": [0-9.e+]*' gpurun_out/r3o/mftopk_b$b.log)"
done
echo ALLDONE
