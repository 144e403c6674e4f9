#!/bin/bash
# Partition chunk per workgroup (FPS_TILE_PARTITION_CHUNK: fewer, longer level-1 / count workgroups
# leave more of the chip to the overlapped SGD), bench.py alternating on one box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/chunk
for rep in 1 2; do
  for c in 65536 131072 262144 524288; do
    FPS_TILE_PARTITION_CHUNK=$c timeout -k 10 200 python bench.py > gpurun_out/chunk/b_$c.$rep.log 2>&1 || { tail -20 gpurun_out/chunk/b_$c.$rep.log; exit 1; }
    python -c "import json; d = json.loads(open('gpurun_out/chunk/b_$c.$rep.log').read().strip().splitlines()[-1]); print('chunk=$c rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
  done
done
