#!/bin/bash
# Adaptive level-3 partition chunk (~16 records per bucket and workgroup) against fixed chunks at the
# per-GPU user counts of the 1-, 4- and 8-GPU configs; tiled tests first.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ca
timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ca/tests.log 2>&1 || { tail -30 gpurun_out/ca/tests.log; exit 1; }
tail -1 gpurun_out/ca/tests.log
for rep in 1 2; do
  for cfg in "10000000 auto" "10000000 65536" "2500000 auto" "2500000 262144" "1250000 auto"; do
    set -- $cfg
    if [ $2 = auto ]; then env=FPS_NONE=1; else env=FPS_TILE_PARTITION_CHUNK=$2; fi
    env $env timeout -k 10 200 python bench.py --users $1 --steps 20 --warmup 3 > gpurun_out/ca/b_$1.$2.$rep.log 2>&1 || { tail -20 gpurun_out/ca/b_$1.$2.$rep.log; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/ca/b_$1.$2.$rep.log').read().strip().splitlines()[-1]); print('users=$1 chunk=$2 rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
  done
done
