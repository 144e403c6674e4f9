#!/bin/bash
# Round 4: virtual-world (RCCL-semantics) GPU tests, then the full GPU validation + Hogwild probe.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b
timeout -k 10 600 python -u -m pytest tests/test_vworld_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4b/vworld.log 2>&1; rc=$?
tail -30 gpurun_out/r4b/vworld.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_vworld_gpu.py > gpurun_out/r4b/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4b/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r4b/bench_n1.log 2>&1 || { tail -20 gpurun_out/r4b/bench_n1.log; exit 1; }
tail -1 gpurun_out/r4b/bench_n1.log | cut -c1-300
timeout -k 10 300 python bench/probe_hogwild.py --phases 1,4 > gpurun_out/r4b/hogwild.log 2>&1 || { tail -20 gpurun_out/r4b/hogwild.log; exit 1; }
cat gpurun_out/r4b/hogwild.log
timeout -k 10 300 python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 4 > gpurun_out/r4b/hogwild_full.log 2>&1 || { tail -20 gpurun_out/r4b/hogwild_full.log; exit 1; }
cat gpurun_out/r4b/hogwild_full.log
echo ALLDONE
