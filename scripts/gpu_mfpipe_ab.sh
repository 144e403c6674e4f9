#!/bin/bash
# A/B of the software-pipelined user-row loads in the tile SGD (FPS_MF_PIPE), same box, alternating
set -e
mkdir -p gpurun_out/mfpipe
FPS_MF_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mfpipe/tests.log 2>&1 || { tail -30 gpurun_out/mfpipe/tests.log; exit 1; }
tail -1 gpurun_out/mfpipe/tests.log
for rep in 1 2; do
  for p in 0 1; do
    FPS_MF_PIPE=$p timeout -k 10 300 python bench.py > gpurun_out/mfpipe/b_${p}_$rep.json 2>/dev/null
    python -c "import json; d=json.loads(open('gpurun_out/mfpipe/b_${p}_$rep.json').read().strip().splitlines()[-1]); print('pipe=$p', d['value'], d['ms_per_step'])"
  done
done
