#!/bin/bash
# A/B of non-temporal streaming accesses in the headline step (FPS_TP_NT: 0 plain, 1 partition
# scatters, 2 + count kernel loads, 3 + the tile SGD's last record read), bench.py alternating
# on one box; the tiled tests at the highest level.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nt
FPS_TP_NT=3 timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nt/tests.log 2>&1 || { tail -30 gpurun_out/nt/tests.log; exit 1; }
tail -1 gpurun_out/nt/tests.log
for rep in 1 2; do
  for v in 0 1 2 3; do
    FPS_TP_NT=$v timeout -k 10 200 python bench.py > gpurun_out/nt/b_$v.$rep.log 2>&1 || { tail -20 gpurun_out/nt/b_$v.$rep.log; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/nt/b_$v.$rep.log').read().strip().splitlines()[-1]); print('nt=$v rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
  done
done
