#!/bin/bash
# Round 3: kernel timeline of the emulated N = 8 rotation step vs N = 1.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3r
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3r/emu8 -- python bench/bench_emulate_world.py --ws 8 --steps 6 --warmup 2 > gpurun_out/r3r/emu8.log 2>&1 || { tail -20 gpurun_out/r3r/emu8.log; exit 1; }
tail -1 gpurun_out/r3r/emu8.log | cut -c1-200
echo ALLDONE
