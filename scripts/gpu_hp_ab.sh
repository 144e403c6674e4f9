#!/bin/bash
# A/B: SGD on a high-priority stream (FPS_SGD_HP=1, default) vs the default stream.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hp
timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hp/tests.log 2>&1 || { tail -20 gpurun_out/hp/tests.log; exit 1; }
tail -1 gpurun_out/hp/tests.log
for v in 0 1 0 1; do
  FPS_SGD_HP=$v timeout -k 10 200 python bench.py > gpurun_out/hp/bench_$v.log 2>&1 || { tail -20 gpurun_out/hp/bench_$v.log; exit 1; }
  echo "hp=$v $(tail -1 gpurun_out/hp/bench_$v.log | cut -c1-160)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hp/prof -- python bench.py --steps 5 --warmup 1 > gpurun_out/hp/prof.log 2>&1 || exit 1
echo ALLDONE
