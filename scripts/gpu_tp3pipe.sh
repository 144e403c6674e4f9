#!/bin/bash
# tp3 scatter register prefetch: tests, same-box A/B (FPS_TP3_PIPE), kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tp3pipe
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tile or tiled" > gpurun_out/tp3pipe/tests.log 2>&1 || { tail -40 gpurun_out/tp3pipe/tests.log; exit 1; }
tail -3 gpurun_out/tp3pipe/tests.log
for rep in 1 2 3; do
  for pp in 0 1; do
    FPS_TP3_PIPE=$pp timeout -k 10 200 python bench.py > gpurun_out/tp3pipe/bench_P${pp}_$rep.log 2>&1 || { tail -20 gpurun_out/tp3pipe/bench_P${pp}_$rep.log; exit 1; }
    echo "PIPE=$pp rep$rep $(tail -1 gpurun_out/tp3pipe/bench_P${pp}_$rep.log | cut -c60-150)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp3pipe/prof_nopf -- python bench.py --steps 5 --warmup 2 --no-prefetch > gpurun_out/tp3pipe/prof_nopf.log 2>&1 || exit 1
FPS_TP3_PIPE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp3pipe/prof_nopf_P0 -- python bench.py --steps 5 --warmup 2 --no-prefetch > gpurun_out/tp3pipe/prof_nopf_P0.log 2>&1 || exit 1
echo ALLDONE
