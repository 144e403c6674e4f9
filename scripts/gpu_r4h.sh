#!/bin/bash
# Round 4 counters: one rocprofv3 --pmc pass per counter group (kernel trace only) over the round-3/4 kernels:
# standard SGNS (sgns_std_kernel / sgns_rows_kernel), the hash-table shard, the request-routing kernel, the bf16
# scorer with COORD on, the MF tile SGD (delta mode, PS path) and the 16-bit partition count kernel.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hogwild_gpu.py tests/test_kernels_gpu.py -k "hogwild or Hogwild or lost or partition or count or 16" -m gpu -x -v --timeout 250 --timeout-method thread > $O/hogwild_tests.log 2>&1 || { tail -30 $O/hogwild_tests.log; exit 1; }
grep -E "PASS|FAIL" $O/hogwild_tests.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
run() {  # name pass cmd...
  name=$1; pass=$2; shift 2
  eval ctr=\$P$pass
  rm -rf $O/${name}_$pass
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${name}_$pass -- "$@" > $O/${name}_$pass.log 2>&1 || { echo "FAIL $name $pass"; tail -5 $O/${name}_$pass.log; exit 1; }
  echo "$name $pass ok"
}
for pass in 1 2 3; do
  run w2v $pass python bench/bench_w2v.py --mode standard --steps 3 --warmup 1 --pairs 1048576
  run hash $pass python bench/probe_kernels.py hash --reps 3
  run route $pass python bench/probe_kernels.py route --reps 3
  run coord $pass python bench/probe_kernels.py coord --reps 2
  run mfps $pass python bench.py --force-ps-path --steps 2 --warmup 1 --no-hogwild-probe
  run emu8 $pass python bench/bench_emulate_world.py --ws 8 --steps 2 --warmup 1
done
python scripts/pmc_summary.py $O w2v,hash,route,coord,mfps,emu8 > $O/summary.md 2>&1 || { cat $O/summary.md; exit 1; }
cat $O/summary.md
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py --steps 6 --warmup 2 > $O/prof_mftopk.log 2>&1 || { tail -20 $O/prof_mftopk.log; exit 1; }
echo ALLDONE
