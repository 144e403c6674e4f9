#!/bin/bash
# GPU pass: tests + MF bench variants (flat / grouped, local / PS-path)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/gpu_tests.log
run() { name=$1; shift; timeout -k 10 200 python bench.py --steps 20 --warmup 3 "$@" > gpurun_out/b_$name.log 2>&1 || { echo "FAIL $name"; exit 1; }; tail -1 gpurun_out/b_$name.log; }
run flat --sgd-mode flat
run grouped --sgd-mode grouped
run grouped16m --sgd-mode grouped --batch 16777216
run ps_flat --sgd-mode flat --force-ps-path
run ps_grouped --sgd-mode grouped --force-ps-path
run ps_grouped_bf16 --sgd-mode grouped --force-ps-path --wire bf16
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/psg -- python bench.py --steps 10 --warmup 2 --sgd-mode grouped --force-ps-path --wire bf16 > gpurun_out/prof_psg.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/lg -- python bench.py --steps 10 --warmup 2 --sgd-mode grouped > gpurun_out/prof_lg.log 2>&1 || exit 1
echo ALLDONE
