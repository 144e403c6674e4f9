#!/bin/bash
# PS-protocol paths through the tensor engine at N = 1 (1 MI355X): MF --force-ps-path, PA, SGNS, capacity
set -e
mkdir -p gpurun_out/pspaths
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --force-ps-path --steps 10 --warmup 3 > gpurun_out/pspaths/mf_ps.log 2>&1 || { tail -20 gpurun_out/pspaths/mf_ps.log; exit 1; }
tail -1 gpurun_out/pspaths/mf_ps.log | cut -c1-300
timeout -k 10 300 python bench/bench_pa.py --ps-path > gpurun_out/pspaths/pa.log 2>&1 || { tail -20 gpurun_out/pspaths/pa.log; exit 1; }
tail -1 gpurun_out/pspaths/pa.log | cut -c1-300
timeout -k 10 300 python bench/bench_w2v.py --ps-path > gpurun_out/pspaths/w2v.log 2>&1 || { tail -20 gpurun_out/pspaths/w2v.log; exit 1; }
tail -1 gpurun_out/pspaths/w2v.log | cut -c1-300
timeout -k 10 300 python bench/bench_capacity.py > gpurun_out/pspaths/cap.log 2>&1 || { tail -20 gpurun_out/pspaths/cap.log; exit 1; }
tail -1 gpurun_out/pspaths/cap.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pspaths/prof_pa -- python bench/bench_pa.py --ps-path --steps 10 > gpurun_out/pspaths/prof_pa.log 2>&1 || { tail -20 gpurun_out/pspaths/prof_pa.log; exit 1; }
