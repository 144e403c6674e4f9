#!/bin/bash
# Round 6 session 3: kernel profile of the online MF + top-K bench (per-batch launch inventory).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3c
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py --steps 20 --warmup 3 > $O/prof_mftopk.log 2>&1 || { tail -20 $O/prof_mftopk.log; exit 1; }
tail -1 $O/prof_mftopk.log | cut -c1-300
echo ALLDONE
