#!/bin/bash
# GPU: w2v + capacity + PA kernel profiles (current code).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 300 python bench/bench_w2v.py > gpurun_out/b_w2v.log 2>&1 || exit 1
tail -1 gpurun_out/b_w2v.log | cut -c1-250
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/w2v -- python bench/bench_w2v.py --steps 5 --warmup 1 > gpurun_out/prof_w2v.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/pa2 -- python bench/bench_pa.py --steps 5 --warmup 1 > gpurun_out/prof_pa2.log 2>&1 || exit 1
echo ALLDONE
