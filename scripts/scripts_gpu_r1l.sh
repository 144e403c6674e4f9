#!/bin/bash
# GPU: tile partition chunk-size sweep (scatter run length vs parallelism).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
for c in 65536 131072 262144 524288; do
  FPS_TILE_PARTITION_CHUNK=$c timeout -k 10 300 python bench.py --steps 20 > gpurun_out/b_chunk$c.log 2>&1 || exit 1
  echo "chunk $c: $(tail -1 gpurun_out/b_chunk$c.log | cut -c60-140)"
done
FPS_TILE_PARTITION_CHUNK=262144 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/chunk262k -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_chunk.log 2>&1 || exit 1
echo ALLDONE
