#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sgk
timeout -k 10 300 python bench/bench_sgns_kernel.py > gpurun_out/sgk/k.log 2>&1 || { tail -20 gpurun_out/sgk/k.log; exit 1; }
grep '^{' gpurun_out/sgk/k.log
echo ALLDONE
