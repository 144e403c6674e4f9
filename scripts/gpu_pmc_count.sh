#!/bin/bash
# PMC passes over the tp3 partition kernels (count / scatter) of the headline MF step.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcc
i=0
for ctr in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmcc/p$i -- python bench.py --steps 2 --warmup 1 --no-prefetch > gpurun_out/pmcc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmcc/p$i.log; exit 1; }
  echo "pass $i ok"
done
echo ALLDONE
