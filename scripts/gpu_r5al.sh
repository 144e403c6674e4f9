#!/bin/bash
# Round 5: bf16 scorer stage of 128 items (st128: half the barriers, 3 waves/SIMD) vs 64 (base).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5al
mkdir -p $O
L=flink_parameter_server_1_amd/_lib
FPS_KERNELS_SO=$L/ab/st128/libfps_kernels.so timeout -k 10 400 python -u -m pytest tests/test_topk_fast.py tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
for r in 1 2; do
  for v in base st128; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    echo "topk $v $r $(tail -1 $O/topk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "mftopk $v $r $(tail -1 $O/mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
for v in base st128; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  export FPS_KERNELS_SO=$so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk_$v -o run -- python bench/bench_topk.py --steps 30 --warmup 3 > $O/prof_topk_$v.log 2>&1 || { tail -20 $O/prof_topk_$v.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk_$v -o run -- python bench/bench_mf_topk.py > $O/prof_mftopk_$v.log 2>&1 || { tail -20 $O/prof_mftopk_$v.log; exit 1; }
  for b in topk mftopk; do
    f=$(find $O/prof_${b}_$v -name "*kernel_stats.csv" | head -1)
    echo "$b $v $(grep score_filter $f | python -c 'import sys,csv; rows=list(csv.reader(sys.stdin)); print(" ".join("%s calls=%s total_ms=%.3f avg_us=%.1f" % (r[0][:50], r[1], float(r[2])/1e6, float(r[3])/1e3) for r in rows))')"
    find $O/prof_${b}_$v -name "*kernel_trace.csv" -delete
  done
done
echo ALLDONE
