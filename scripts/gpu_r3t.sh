#!/bin/bash
# Round 3: top-K merge: threshold refined to <= TK_NT candidates, wave-aggregated histogram + slots (B = tree) vs HEAD (A = _lib/ab), same box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3t
timeout -k 10 600 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "topk or lemp or merge" > gpurun_out/r3t/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3t/tests.log
[ $rc -eq 0 ] || exit 1
A=$GRAFT_REPO_ROOT/flink_parameter_server_1_amd/_lib/ab/libfps_kernels_a.so
for rep in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export FPS_KERNELS_SO=$A; else unset FPS_KERNELS_SO; fi
    timeout -k 10 300 python bench/bench_topk.py > gpurun_out/r3t/topk_$v$rep.log 2>&1 || { tail -20 gpurun_out/r3t/topk_$v$rep.log; exit 1; }
    timeout -k 10 300 python bench/bench_mf_topk.py > gpurun_out/r3t/mftopk_$v$rep.log 2>&1 || { tail -20 gpurun_out/r3t/mftopk_$v$rep.log; exit 1; }
    echo "$v$rep topk $(grep -o '"value": [0-9.e+]*' gpurun_out/r3t/topk_$v$rep.log) $(grep -o '"exact_vs_brute_force": [a-z]*' gpurun_out/r3t/topk_$v$rep.log) mftopk $(grep -o '"value": [0-9.e+]*' gpurun_out/r3t/mftopk_$v$rep.log)"
  done
done
unset FPS_KERNELS_SO
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3t/prof_topk -- python bench/bench_topk.py --steps 10 > gpurun_out/r3t/prof.log 2>&1 || { tail -20 gpurun_out/r3t/prof.log; exit 1; }
echo ALLDONE
