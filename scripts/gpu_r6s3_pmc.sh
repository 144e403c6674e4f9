#!/bin/bash
# Round 6 session 3: PMC passes over the headline's timed loop on the final build (prefetch side stream on, as timed):
# pass 1 SQ counters + GRBM, pass 2 FETCH_SIZE, pass 3 WRITE_SIZE (one counter group per run, kernel trace only).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3pmc
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for ctr in "$P1" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  rm -rf $O/mf_$i
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/mf_$i -- python bench.py --steps 5 --warmup 2 --no-hogwild-probe --exact-steps 0 > $O/mf_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/mf_$i.log; exit 1; }
  echo "pass $i ok"
done
python scripts/pmc_summary.py $O mf 6
echo ALLDONE
