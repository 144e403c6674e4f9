#!/bin/bash
# GPU: tile rows sweep x prefetch on/off (same box, A/B).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
for R in 64 128 256; do
  for c in 65536 262144; do
    FPS_TILE_ROWS=$R FPS_TILE_PARTITION_CHUNK=$c timeout -k 10 300 python bench.py --steps 20 > gpurun_out/b_R${R}_c$c.log 2>&1 || exit 1
    echo "R=$R chunk=$c: $(tail -1 gpurun_out/b_R${R}_c$c.log | cut -c60-150)"
  done
done
FPS_TILE_ROWS=256 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/R256 -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_R256.log 2>&1 || exit 1
echo ALLDONE
