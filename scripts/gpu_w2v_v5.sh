#!/bin/bash
# SGNS kernel v5 (loader / atomic wave split): numerics vs reference, bench v4 vs v5, kernel stats, PMC.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w2v5
timeout -k 10 300 python -u -m pytest tests/test_sgns_sampling.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/w2v5/tests.log 2>&1 || { tail -30 gpurun_out/w2v5/tests.log; exit 1; }
tail -1 gpurun_out/w2v5/tests.log
for K in v4 v5; do
  FPS_SGNS_KERNEL=$K timeout -k 10 300 python bench/bench_w2v.py > gpurun_out/w2v5/bench_$K.log 2>&1 || { tail -20 gpurun_out/w2v5/bench_$K.log; exit 1; }
  echo "$K $(grep '^{' gpurun_out/w2v5/bench_$K.log | cut -c60-330)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w2v5/prof -- python bench/bench_w2v.py --steps 8 --warmup 2 > gpurun_out/w2v5/prof.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/w2v5/pmc1 -- python bench/bench_w2v.py --steps 2 --warmup 1 > gpurun_out/w2v5/pmc1.log 2>&1 || { echo pmc1 failed; tail -3 gpurun_out/w2v5/pmc1.log; }
echo ALLDONE
