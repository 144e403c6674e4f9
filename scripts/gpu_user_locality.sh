#!/bin/bash
# Experiment: tiled MF SGD kernel time vs the size of the user id range (MALL reuse of user rows).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/loc
for U in 250000 500000 1000000 2000000 10000000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/loc/u$U -- python bench.py --steps 4 --warmup 1 --users $U --no-prefetch > gpurun_out/loc/u$U.log 2>&1 || exit 1
  tail -1 gpurun_out/loc/u$U.log | cut -c1-140
done
echo ALLDONE
