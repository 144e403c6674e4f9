#!/bin/bash
# A/B of non-temporal item-row accesses in the tile SGD (FPS_SGD_NT=0: plain; default: non-temporal),
# bench.py alternating on one box.  (The user-row variants of profiles/r2_partition.md were an A/B
# patch, not kept: no gain.)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/snt
for v in 0 1; do
  FPS_SGD_NT=$v timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/snt/tests_$v.log 2>&1 || { tail -30 gpurun_out/snt/tests_$v.log; exit 1; }
done
for rep in 1 2; do
  for v in 0 1; do
    FPS_SGD_NT=$v timeout -k 10 200 python bench.py > gpurun_out/snt/b_$v.$rep.log 2>&1 || { tail -20 gpurun_out/snt/b_$v.$rep.log; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/snt/b_$v.$rep.log').read().strip().splitlines()[-1]); print('sgd_nt=$v rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
  done
done
