#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ba
mkdir -p $O
timeout -k 10 300 python bench/diag_pa_ops.py > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
timeout -k 10 300 python bench/bench_pa.py --ps-path > $O/pa.log 2>&1 || { tail -20 $O/pa.log; exit 1; }
tail -1 $O/pa.log | cut -c1-300
echo ALLDONE
