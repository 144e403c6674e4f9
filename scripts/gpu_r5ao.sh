#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ao
mkdir -p $O
timeout -k 10 300 python bench/diag_mf_topk_ops.py > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
echo ALLDONE
