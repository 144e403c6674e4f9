#!/bin/bash
# A/B of the level-1 record layout under the non-temporal policy (FPS_TP_NT: 0 plain 12-B records
# = the round's earlier code, 1 non-temporal 12-B records as three dwords, 2 non-temporal 12-B
# records in 16-B slots), bench.py alternating on one box; tiled tests for modes 0 and 1.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nt2
for v in 0 1; do
  FPS_TP_NT=$v timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nt2/tests_$v.log 2>&1 || { tail -30 gpurun_out/nt2/tests_$v.log; exit 1; }
done
for rep in 1 2 3; do
  for v in 0 1 2; do
    FPS_TP_NT=$v timeout -k 10 200 python bench.py > gpurun_out/nt2/b_$v.$rep.log 2>&1 || { tail -20 gpurun_out/nt2/b_$v.$rep.log; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/nt2/b_$v.$rep.log').read().strip().splitlines()[-1]); print('tp_nt=$v rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
  done
done
