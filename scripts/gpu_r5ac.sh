#!/bin/bash
# Round 5: kernel traces of the local headline and the fused MF PS path (same box) for a timeline comparison.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ac
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/local -- python bench.py --steps 6 --warmup 2 --no-hogwild-probe > $O/local.log 2>&1 || { tail -20 $O/local.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ps -- python bench.py --steps 6 --warmup 2 --force-ps-path --no-hogwild-probe > $O/ps.log 2>&1 || { tail -20 $O/ps.log; exit 1; }
echo ALLDONE
