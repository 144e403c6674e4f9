#!/bin/bash
# Round 3: kernel stats + timeline of standard SGNS through the PS path.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3v
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3v/prof -- python bench/bench_w2v.py --mode standard --ps-path --steps 6 --warmup 2 > gpurun_out/r3v/w2v.log 2>&1 || { tail -20 gpurun_out/r3v/w2v.log; exit 1; }
tail -1 gpurun_out/r3v/w2v.log | cut -c1-150
echo ALLDONE
