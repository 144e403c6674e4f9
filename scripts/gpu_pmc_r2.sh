#!/bin/bash
# Round-2 PMC passes (one counter group per run; no trace domains besides kernel-trace)
# over the three hot paths: MF+top-K serving (score_filter), SGNS v4 (negative groups),
# the headline MF step without prefetch (tile SGD + partition).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
run() {  # name pass counters -- cmd...
  local name=$1 pass=$2 ctr=$3; shift 3
  rm -rf gpurun_out/pmc/${name}_$pass
  timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc/${name}_$pass -- "$@" > gpurun_out/pmc/${name}_$pass.log 2>&1
  echo "$name $pass ok"
}
for pass in 1 2 3; do
  eval ctr=\$P$pass
  run mftopk $pass "$ctr" python bench/bench_mf_topk.py --steps 4 --warmup 1
  run w2v $pass "$ctr" python bench/bench_w2v.py --steps 4 --warmup 1
  run mf $pass "$ctr" python bench.py --steps 3 --warmup 1 --no-prefetch
done
