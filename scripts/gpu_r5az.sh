#!/bin/bash
# Round 5 end: per-GPU step of the N = 1/2/4/8 rotation (rank 0's schedule emulated on one GPU), final build,
# default user-row mode (exact at N > 1) and Hogwild for reference.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5az
mkdir -p $O
timeout -k 10 500 python bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3 > $O/auto.log 2>&1 || { tail -20 $O/auto.log; exit 1; }
grep '^{' $O/auto.log | cut -c1-400
timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 10 --warmup 3 --user-update store > $O/store8.log 2>&1 || { tail -20 $O/store8.log; exit 1; }
grep '^{' $O/store8.log | cut -c1-400
echo ALLDONE
