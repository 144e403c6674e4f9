#!/bin/bash
set -e
mkdir -p gpurun_out/engine
timeout -k 10 300 python bench/bench_engine.py > gpurun_out/engine/s0.json && cat gpurun_out/engine/s0.json
timeout -k 10 300 python bench/bench_engine.py --staleness 1 > gpurun_out/engine/s1.json && cat gpurun_out/engine/s1.json
rm -rf gpurun_out/engine/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/engine/prof -- python bench/bench_engine.py --batches 64 --seconds 1 > gpurun_out/engine/prof.log 2>&1
