#!/bin/bash
# Round 3: kernel stats of the top-K scan (bench_topk length) and the MF + top-K serving bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3l
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3l/prof_topk -- python bench/bench_topk.py --steps 10 > gpurun_out/r3l/topk.log 2>&1 || { tail -20 gpurun_out/r3l/topk.log; exit 1; }
tail -1 gpurun_out/r3l/topk.log | cut -c1-150
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3l/prof_mftopk -- python bench/bench_mf_topk.py > gpurun_out/r3l/mftopk.log 2>&1 || { tail -20 gpurun_out/r3l/mftopk.log; exit 1; }
tail -1 gpurun_out/r3l/mftopk.log | cut -c1-150
echo ALLDONE
