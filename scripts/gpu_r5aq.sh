#!/bin/bash
# Round 5: scorer with all MFMA chains of a block pair issued before their filters (ilv) vs one chain + filter at a time (base).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5aq
mkdir -p $O
L=flink_parameter_server_1_amd/_lib
for v in ilv; do
  FPS_KERNELS_SO=$L/ab/$v/libfps_kernels.so timeout -k 10 400 python -u -m pytest tests/test_topk_fast.py tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "tests $v $(tail -1 $O/tests_$v.log)"
done
for r in 1 2; do
for v in base ilv; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  export FPS_KERNELS_SO=$so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk_${v}_$r -o run -- python bench/bench_topk.py --steps 30 --warmup 3 > $O/prof_topk_${v}_$r.log 2>&1 || { tail -20 $O/prof_topk_${v}_$r.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk_${v}_$r -o run -- python bench/bench_mf_topk.py > $O/prof_mftopk_${v}_$r.log 2>&1 || { tail -20 $O/prof_mftopk_${v}_$r.log; exit 1; }
  for b in topk mftopk; do
    f=$(find $O/prof_${b}_${v}_$r -name "*kernel_stats.csv" | head -1)
    echo "$b $v $r $(tail -1 $O/prof_${b}_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])') $(grep "score_filter\|merge_rank" $f | python -c 'import sys,csv; rows=list(csv.reader(sys.stdin)); print(" ".join("%s=%.3fms" % (r[0].split("(")[0].split("::")[-1][:28], float(r[2])/1e6) for r in rows))')"
    find $O/prof_${b}_${v}_$r -name "*kernel_trace.csv" -delete
  done
done
done
echo ALLDONE
