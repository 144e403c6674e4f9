#!/bin/bash
# Round 3: PA PS path after the touched-mark changes (tests of the PS / contract paths, bench, kernel trace).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3j
timeout -k 10 600 python -u -m pytest tests/test_tensor_engine_gpu.py tests/test_tensor_contract_gpu.py tests/test_kernels_gpu.py tests/test_pa_offline_tensor_gpu.py tests/test_pa_fast.py tests/test_pa_reference_scale.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3j/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3j/tests.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench/bench_pa.py --ps-path > gpurun_out/r3j/pa_ps$rep.log 2>&1 || { tail -20 gpurun_out/r3j/pa_ps$rep.log; exit 1; }
  tail -1 gpurun_out/r3j/pa_ps$rep.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3j/prof_pa -- python bench/bench_pa.py --ps-path --steps 5 --warmup 1 > gpurun_out/r3j/prof_pa.log 2>&1 || { tail -20 gpurun_out/r3j/prof_pa.log; exit 1; }
echo ALLDONE
