#!/bin/bash
# GPU profiling pass: kernel stats + PMC counters for the MF bench (1 GPU)
set -o pipefail
export TMPDIR=/tmp
cd /tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 300 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/gpu_tests.log
for B in 1048576 4194304 16777216; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --batch $B > gpurun_out/bench_b$B.log 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --user-update atomic > gpurun_out/bench_atomic.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -- python bench.py --steps 10 --warmup 2 > gpurun_out/prof_kt.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc1 -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_pmc1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof/pmc2 -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_pmc2.log 2>&1 || exit 1
echo ALLDONE
