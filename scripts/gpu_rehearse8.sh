#!/bin/bash
# 8 ranks sharing one MI355X over gloo: bench.py's N = 8 code path (tiled SGD, 16-block ring
# rotation, user phases) end to end at small shapes
set -e
mkdir -p gpurun_out/rehearse
export TMPDIR=/tmp FPS_SHARE_GPU=1
timeout -k 10 400 python bench.py --gpus 8 --steps 3 --warmup 1 --batch 1048576 --users 2000000 > gpurun_out/rehearse/share8.log 2>&1 || { tail -30 gpurun_out/rehearse/share8.log; exit 1; }
tail -1 gpurun_out/rehearse/share8.log | cut -c1-400
