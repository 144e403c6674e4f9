#!/bin/bash
# Partition chunk (FPS_TILE_PARTITION_CHUNK) at the per-GPU user counts of the 4- and 8-GPU configs.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cu
for rep in 1 2; do
  for u in 2500000 1250000; do
    for c in 65536 262144; do
      FPS_TILE_PARTITION_CHUNK=$c timeout -k 10 200 python bench.py --users $u --steps 20 --warmup 3 > gpurun_out/cu/b_$u.$c.$rep.log 2>&1 || { tail -20 gpurun_out/cu/b_$u.$c.$rep.log; exit 1; }
      python -c "import json; d = json.loads(open('gpurun_out/cu/b_$u.$c.$rep.log').read().strip().splitlines()[-1]); print('users=$u chunk=$c rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
    done
  done
done
