#!/bin/bash
# PMC passes over the tiled MF step (one pass per counter group, kernel trace only).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/p$i -- python bench.py --steps 2 --warmup 1 --no-prefetch > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok"
done
echo ALLDONE
