#!/bin/bash
# Round 4: Hogwild A/B (user rows plain vs write-through sc1), virtual-world N = 8 diagnosis, HW-queue A/B.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py -m gpu -x -q -k "tiled" --timeout 150 --timeout-method thread > gpurun_out/r4e/tiled_tests.log 2>&1 || { tail -30 gpurun_out/r4e/tiled_tests.log; exit 1; }
tail -1 gpurun_out/r4e/tiled_tests.log
FPS_MF_USER_SC1=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py -m gpu -x -q -k "tiled and not converge and not matches_synchronous" --timeout 150 --timeout-method thread > gpurun_out/r4e/tiled_tests_sc1.log 2>&1 || { tail -30 gpurun_out/r4e/tiled_tests_sc1.log; exit 1; }
tail -1 gpurun_out/r4e/tiled_tests_sc1.log
for mode in 0 1; do
  FPS_MF_USER_SC1=$mode timeout -k 10 300 python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 1,4 > gpurun_out/r4e/hogwild_sc1_$mode.log 2>&1 || { tail -20 gpurun_out/r4e/hogwild_sc1_$mode.log; exit 1; }
  echo "sc1=$mode"; cat gpurun_out/r4e/hogwild_sc1_$mode.log | grep users
  FPS_MF_USER_SC1=$mode timeout -k 10 300 python bench.py > gpurun_out/r4e/bench_sc1_$mode.log 2>&1 || { tail -20 gpurun_out/r4e/bench_sc1_$mode.log; exit 1; }
  tail -1 gpurun_out/r4e/bench_sc1_$mode.log | cut -c1-200
done
FPS_MF_USER_SC1=1 timeout -k 10 300 python bench.py > gpurun_out/r4e/bench_sc1_1b.log 2>&1 || { tail -20 gpurun_out/r4e/bench_sc1_1b.log; exit 1; }
tail -1 gpurun_out/r4e/bench_sc1_1b.log | cut -c1-200
timeout -k 10 200 python -u bench/bench_vworld.py --world 8 --batch 4194304 --steps 3 --warmup 1 --traceback-s 45 > gpurun_out/r4e/vworld_n8_small.log 2>&1; rc=$?
tail -5 gpurun_out/r4e/vworld_n8_small.log
[ $rc -eq 0 ] || { echo "n8 small rc=$rc"; exit 1; }
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python -u bench/bench_vworld.py --world 4 --traceback-s 60 > gpurun_out/r4e/vworld_n4_q16.log 2>&1 || { tail -20 gpurun_out/r4e/vworld_n4_q16.log; exit 1; }
tail -1 gpurun_out/r4e/vworld_n4_q16.log
echo ALLDONE
