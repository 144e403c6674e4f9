#!/bin/bash
# Round 5: seen merge with the sorted-input compaction (default) vs the sort for every row (sm0 = HEAD).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5as
mkdir -p $O
L=flink_parameter_server_1_amd/_lib
timeout -k 10 400 python -u -m pytest tests/test_topk_seen_merge_gpu.py tests/test_topk_tensor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
for r in 1 2; do
for v in base sm0; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  export FPS_KERNELS_SO=$so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk_${v}_$r -o run -- python bench/bench_mf_topk.py > $O/prof_mftopk_${v}_$r.log 2>&1 || { tail -20 $O/prof_mftopk_${v}_$r.log; exit 1; }
  f=$(find $O/prof_mftopk_${v}_$r -name "*kernel_stats.csv" | head -1)
  echo "mftopk $v $r $(grep '^{' $O/prof_mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])') $(grep "seen_merge" $f | python -c 'import sys,csv; rows=list(csv.reader(sys.stdin)); print(" ".join("seen_merge calls=%s total_ms=%.3f avg_us=%.1f" % (r[1], float(r[2])/1e6, float(r[3])/1e3) for r in rows))')"
  find $O/prof_mftopk_${v}_$r -name "*kernel_trace.csv" -delete
done
done
echo ALLDONE
