#!/bin/bash
# SGNS negative groups: kernel numerics vs the reference, then bench_w2v at groups 1 / 2 / 4 (alternating)
set -e
mkdir -p gpurun_out/sgns
timeout -k 10 400 python -u -m pytest tests/test_sgns_sampling.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sgns/tests.log 2>&1 || { tail -30 gpurun_out/sgns/tests.log; exit 1; }
tail -1 gpurun_out/sgns/tests.log
for rep in 1 2; do
  for g in 1 2 4; do
    timeout -k 10 200 python bench/bench_w2v.py --neg-group $g > gpurun_out/sgns/w2v_g${g}_r$rep.json 2>&1 || { tail -20 gpurun_out/sgns/w2v_g${g}_r$rep.json; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('loss_first_last'))" gpurun_out/sgns/w2v_g${g}_r$rep.json g$g
  done
done
