#!/bin/bash
# Refresh secondary numbers after the tiled-SGD staging changes: PS path (forced), rotation sub-step shapes.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/refresh
timeout -k 10 300 python bench.py --force-ps-path --steps 10 --warmup 2 > gpurun_out/refresh/ps.log 2>&1 || { tail -20 gpurun_out/refresh/ps.log; exit 1; }
echo "ps $(grep '^{' gpurun_out/refresh/ps.log | cut -c80-200)"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/refresh/n1.log 2>&1 || { tail -20 gpurun_out/refresh/n1.log; exit 1; }
echo "n1 $(grep '^{' gpurun_out/refresh/n1.log | cut -c80-200)"
timeout -k 10 400 python bench/bench_tiled_substeps.py > gpurun_out/refresh/sub.log 2>&1 || { tail -20 gpurun_out/refresh/sub.log; exit 1; }
grep '^{' gpurun_out/refresh/sub.log
echo ALLDONE
