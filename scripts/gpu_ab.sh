#!/bin/bash
# A/B of two kernel-library builds (ab/libA.so, ab/libB.so) on one box: headline bench, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
for V in A B; do
  FPS_KERNELS_SO=$PWD/ab/lib$V.so timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ab/b_$V.log 2>&1 || { tail -20 gpurun_out/ab/b_$V.log; exit 1; }
  echo "$V $(grep '^{' gpurun_out/ab/b_$V.log | cut -c80-200)"
done
done
echo ALLDONE
