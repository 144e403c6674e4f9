#!/bin/bash
# Round 5: seed-select occupancy (3 waves per SIMD, 168 VGPRs, vs the unconstrained 197: variant ts2) and scorer floor
# 512 / 768 / 1024 -- LEMP, alternating; select-kernel tests.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5w
mkdir -p $O
L=$PWD/flink_parameter_server_1_amd/_lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "topk_select" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base ts2; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    echo "topk $v $r $(tail -1 $O/topk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
  done
  for m in 512 768; do
    FPS_SB_MIN_WGS=$m timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_m${m}_$r.log 2>&1 || { tail -20 $O/topk_m${m}_$r.log; exit 1; }
    echo "topk minwgs=$m $r $(tail -1 $O/topk_m${m}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk -- python bench/bench_topk.py --steps 20 --warmup 3 > $O/prof_topk.log 2>&1 || { tail -20 $O/prof_topk.log; exit 1; }
echo ALLDONE
