#!/bin/bash
# A/B: partition / SGD on disjoint CU sets (FPS_PARTITION_CUS), alternating on one box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cumask
timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "prefetch or exact" > gpurun_out/cumask/tests.log 2>&1 || { tail -30 gpurun_out/cumask/tests.log; exit 1; }
FPS_PARTITION_CUS=32 timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "prefetch or exact" >> gpurun_out/cumask/tests.log 2>&1 || { tail -30 gpurun_out/cumask/tests.log; exit 1; }
tail -2 gpurun_out/cumask/tests.log
for rep in 1 2; do
  for k in 0 16 32 64; do
    FPS_PARTITION_CUS=$k timeout -k 10 200 python bench.py > gpurun_out/cumask/bench_${k}_$rep.log 2>&1 || { tail -20 gpurun_out/cumask/bench_${k}_$rep.log; exit 1; }
    echo "CUS=$k rep$rep $(tail -1 gpurun_out/cumask/bench_${k}_$rep.log | cut -c60-160)"
  done
done
echo ALLDONE
