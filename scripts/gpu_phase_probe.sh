#!/bin/bash
# Probe: would user phases (MALL-sized user ranges per SGD launch) pay?  A phase of a
# 64M-rating step at P phases = a 64M/P-rating step over 10M/P users.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/phase
for cfg in "10000000 67108864" "2500000 16777216" "1250000 8388608" "5000000 33554432"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/phase/u$1 -- python bench.py --steps 8 --warmup 2 --users $1 --batch $2 --no-prefetch > gpurun_out/phase/u$1.log 2>&1 || exit 1
  echo "$1 $2 $(grep '^{' gpurun_out/phase/u$1.log | cut -c80-200)"
done
echo ALLDONE
