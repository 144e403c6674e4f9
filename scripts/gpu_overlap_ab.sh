#!/bin/bash
# Overlap modes with the final partition defaults: side-stream prefetch (default), serial
# (--no-prefetch), SGD on a priority stream (--sgd-high-priority); bench.py alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ov
for rep in 1 2; do
  for v in default no-prefetch sgd-high-priority; do
    flag=""; [ $v != default ] && flag="--$v"
    timeout -k 10 200 python bench.py $flag > gpurun_out/ov/b_$v.$rep.log 2>&1 || { tail -20 gpurun_out/ov/b_$v.$rep.log; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/ov/b_$v.$rep.log').read().strip().splitlines()[-1]); print('$v rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
  done
done
