#!/bin/bash
# User phases per step (--user-phases) with the non-temporal partition / item rows, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ph
for rep in 1 2; do
  for p in 2 3 4; do
    timeout -k 10 200 python bench.py --user-phases $p > gpurun_out/ph/b_$p.$rep.log 2>&1 || { tail -20 gpurun_out/ph/b_$p.$rep.log; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/ph/b_$p.$rep.log').read().strip().splitlines()[-1]); print('phases=$p rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
  done
done
