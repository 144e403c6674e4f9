#!/bin/bash
# Round 5: the LDS-staged bf16 scorer -- top-K GPU tests, same-box A/B against the previous scorer (LEMP top-100
# and online MF + top-K), and one counter pass over the scorer.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5e
mkdir -p $O
L=$PWD/flink_parameter_server_1_amd/_lib
timeout -k 10 600 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_seen_merge_gpu.py tests/test_topk_tensor_gpu.py tests/test_topk_fast.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for v in new sbold; do
    so=$L/libfps_kernels.so; [ $v = sbold ] && so=$L/ab/sbold/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_topk.py > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "$v $r topk $(tail -1 $O/topk_${v}_$r.log | cut -c1-120) | mftopk $(tail -1 $O/mftopk_${v}_$r.log | cut -c1-120)"
  done
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for v in new sbold; do
  so=$L/libfps_kernels.so; [ $v = sbold ] && so=$L/ab/sbold/libfps_kernels.so
  rm -rf $O/pmc_$v
  FPS_KERNELS_SO=$so timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/pmc_$v -- python bench/bench_topk.py --steps 5 --warmup 1 > $O/pmc_$v.log 2>&1 || { echo "FAIL pmc $v"; tail -5 $O/pmc_$v.log; exit 1; }
  echo "pmc $v ok"
done
echo ALLDONE
