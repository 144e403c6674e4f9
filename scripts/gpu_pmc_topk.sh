#!/bin/bash
# PMC passes of the bf16 top-K scan (bench/bench_topk.py and bench/bench_mf_topk.py): one counter
# group per run (kernel-trace only), then the per-kernel summary of scripts/pmc_summary.py.
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmct
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
for pass in 1 2 3; do
  eval ctr=\$P$pass
  for name in topk mftopk; do
    rm -rf gpurun_out/pmct/${name}_$pass
    script=bench/bench_topk.py; [ $name = mftopk ] && script=bench/bench_mf_topk.py
    timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmct/${name}_$pass -- python $script --steps 4 --warmup 1 > gpurun_out/pmct/${name}_$pass.log 2>&1
    echo "$name $pass ok"
  done
done
