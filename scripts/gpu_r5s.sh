#!/bin/bash
# Round 5: kernel stats of MF + top-K with the current kernels vs the "preload" variant (one commit earlier)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5s
mkdir -p $O
L=$PWD/flink_parameter_server_1_amd/_lib
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_base -- python bench/bench_mf_topk.py > $O/base.log 2>&1 || { tail -20 $O/base.log; exit 1; }
FPS_KERNELS_SO=$L/ab/preload/libfps_kernels.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_preload -- python bench/bench_mf_topk.py > $O/preload.log 2>&1 || { tail -20 $O/preload.log; exit 1; }
echo ALLDONE
