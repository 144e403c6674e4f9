#!/bin/bash
# A/B: partition prefetch on a side stream (default) vs serial (--no-prefetch), alternating on one box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pfab
for rep in 1 2 3; do
  for mode in pf nopf; do
    flag=""; [ $mode = nopf ] && flag="--no-prefetch"
    timeout -k 10 200 python bench.py $flag > gpurun_out/pfab/bench_${mode}_$rep.log 2>&1 || { tail -20 gpurun_out/pfab/bench_${mode}_$rep.log; exit 1; }
    echo "$mode rep$rep $(tail -1 gpurun_out/pfab/bench_${mode}_$rep.log | cut -c60-175)"
  done
done
echo ALLDONE
