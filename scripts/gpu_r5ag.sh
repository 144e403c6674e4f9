#!/bin/bash
# Round 5: scorer epilogue (filter all query blocks, then emit) and 2 query blocks per
# wave (4 waves / SIMD) vs the default -- correctness, then LEMP and MF + top-K A/B, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ag
mkdir -p $O
L=flink_parameter_server_1_amd/_lib
for v in epi1 qb2 epi1qb2; do
  FPS_KERNELS_SO=$L/ab/$v/libfps_kernels.so timeout -k 10 300 python -u -m pytest tests/test_topk_bf16_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_$v.log 2>&1 || { tail -30 $O/test_$v.log; exit 1; }
  echo "tests $v $(tail -1 $O/test_$v.log)"
done
for r in 1 2; do
  for v in base epi1 qb2 epi1qb2; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    echo "topk $v $r $(tail -1 $O/topk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "mftopk $v $r $(tail -1 $O/mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
echo ALLDONE
