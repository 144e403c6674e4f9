#!/bin/bash
# A/B: tiled SGD on a high-priority stream (bench.py --sgd-high-priority) vs the default stream.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hp
for v in off on; do
  flag=""; [ $v = on ] && flag="--sgd-high-priority"
  timeout -k 10 200 python bench.py $flag > gpurun_out/hp/bench_$v.log 2>&1 || { tail -20 gpurun_out/hp/bench_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/hp/bench_$v.log | cut -c1-200)"
done
