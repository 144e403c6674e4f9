#!/bin/bash
set -e
mkdir -p gpurun_out/mfps
export TMPDIR=/tmp
rm -rf gpurun_out/mfps/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mfps/prof -- python bench.py --force-ps-path --steps 10 --warmup 3 > gpurun_out/mfps/prof.log 2>&1 || { tail -20 gpurun_out/mfps/prof.log; exit 1; }
tail -1 gpurun_out/mfps/prof.log | cut -c1-200
