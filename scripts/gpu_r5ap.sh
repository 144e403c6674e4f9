#!/bin/bash
# Round 5: PMC counters of the final top-K build (scorer at 2 query blocks per wave, re-score and rank-merge loads issued first).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ap
mkdir -p $O
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
  run topk $pass python bench/bench_topk.py --steps 6 --warmup 2
  run mftopk $pass python bench/bench_mf_topk.py
done
python scripts/pmc_summary.py $O topk,mftopk 8 > $O/summary.md 2>&1 || { cat $O/summary.md; exit 1; }
cat $O/summary.md
echo ALLDONE
