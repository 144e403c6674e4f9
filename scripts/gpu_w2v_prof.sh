#!/bin/bash
# SGNS (BASELINE config #3): bench line, kernel stats, one PMC pass.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w2v
timeout -k 10 300 python bench/bench_w2v.py > gpurun_out/w2v/bench.log 2>&1 || { tail -20 gpurun_out/w2v/bench.log; exit 1; }
grep '^{' gpurun_out/w2v/bench.log | cut -c1-250
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w2v/prof -- python bench/bench_w2v.py --steps 8 --warmup 2 > gpurun_out/w2v/prof.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/w2v/pmc1 -- python bench/bench_w2v.py --steps 2 --warmup 1 > gpurun_out/w2v/pmc1.log 2>&1 || { echo pmc1 failed; tail -3 gpurun_out/w2v/pmc1.log; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/w2v/pmc2 -- python bench/bench_w2v.py --steps 2 --warmup 1 > gpurun_out/w2v/pmc2.log 2>&1 || { echo pmc2 failed; tail -3 gpurun_out/w2v/pmc2.log; }
echo ALLDONE
