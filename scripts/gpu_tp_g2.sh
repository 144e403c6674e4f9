#!/bin/bash
# Level-2 scatter workgroups (FPS_TP3_G2 cap; they loop over the work items), bench.py alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g2
for rep in 1 2; do
  for g in 1024 512 256; do
    FPS_TP3_G2=$g timeout -k 10 200 python bench.py > gpurun_out/g2/b_$g.$rep.log 2>&1 || { tail -20 gpurun_out/g2/b_$g.$rep.log; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/g2/b_$g.$rep.log').read().strip().splitlines()[-1]); print('g2=$g rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
  done
done
