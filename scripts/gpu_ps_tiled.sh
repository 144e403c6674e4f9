#!/bin/bash
# PS (pull/push) path with the tile-grouped SGD on the pulled rows: tests, bench vs flat, kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pst
timeout -k 10 400 python -u -m pytest tests/test_kernels_grouped_gpu.py tests/test_multirank_gpu.py tests/test_mf_tiled_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pst/tests.log 2>&1 || { tail -30 gpurun_out/pst/tests.log; exit 1; }
tail -1 gpurun_out/pst/tests.log
for M in flat tiled; do
  timeout -k 10 300 python bench.py --force-ps-path --sgd-mode $M --steps 10 --warmup 2 > gpurun_out/pst/b_$M.log 2>&1 || { tail -20 gpurun_out/pst/b_$M.log; exit 1; }
  echo "$M $(grep '^{' gpurun_out/pst/b_$M.log | cut -c80-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pst/prof -- python bench.py --force-ps-path --steps 5 --warmup 1 > gpurun_out/pst/prof.log 2>&1 || exit 1
echo ALLDONE
