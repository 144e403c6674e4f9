#!/bin/bash
# Round 5: scorer cost breakdown (timing-only diagnostic builds: noemit = no score passes the filter,
# nomfma = no MFMA; both give wrong top-K results) -- kernel totals of the scorer.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ar
mkdir -p $O
L=flink_parameter_server_1_amd/_lib
for v in base noemit; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  export FPS_KERNELS_SO=$so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk_$v -o run -- python bench/bench_topk.py --steps 30 --warmup 3 > $O/prof_topk_$v.log 2>&1
  echo "topk $v rc=$? $(grep score_filter $(find $O/prof_topk_$v -name '*kernel_stats.csv' | head -1) | python -c 'import sys,csv; rows=list(csv.reader(sys.stdin)); print(" ".join("calls=%s total_ms=%.3f" % (r[1], float(r[2])/1e6) for r in rows))')"
  find $O/prof_topk_$v -name "*kernel_trace.csv" -delete
done
echo ALLDONE
