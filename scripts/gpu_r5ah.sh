#!/bin/bash
# Round 5: scorer kernel time, 4 vs 2 query blocks per wave (rocprofv3 --stats)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ah
mkdir -p $O
L=flink_parameter_server_1_amd/_lib
for r in 1 2; do
for v in base qb2; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  export FPS_KERNELS_SO=$so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/topk_${v}_$r -o run -- python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mftopk_${v}_$r -o run -- python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
  for b in topk mftopk; do
    f=$(find $O/${b}_${v}_$r -name "*kernel_stats.csv" | head -1)
    echo "$b $v $r $(grep score_filter $f | python -c 'import sys,csv; rows=list(csv.reader(sys.stdin)); print(" ".join("%s calls=%s total_ms=%.3f" % (r[0][:60], r[1], float(r[2])/1e6) for r in rows))')"
    find $O/${b}_${v}_$r -name "*kernel_trace.csv" -delete
  done
done
done
echo ALLDONE
