#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/gpu_tests.log
run() { name=$1; shift; timeout -k 10 200 python bench.py --steps 20 --warmup 3 "$@" > gpurun_out/b_$name.log 2>&1 || { echo "FAIL $name"; exit 1; }; tail -1 gpurun_out/b_$name.log | cut -c1-200; }
run default
run ps_flat --sgd-mode flat --force-ps-path
run ps_grouped --sgd-mode grouped --force-ps-path
run ps_flat_bf16 --sgd-mode flat --force-ps-path --wire bf16
timeout -k 10 300 python bench/bench_w2v.py --steps 10 --warmup 2 > gpurun_out/b_w2v.log 2>&1 || { echo FAIL w2v; exit 1; }
tail -1 gpurun_out/b_w2v.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/psf -- python bench.py --steps 10 --warmup 2 --sgd-mode flat --force-ps-path > gpurun_out/prof_psf.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/w2v -- python bench/bench_w2v.py --steps 5 --warmup 1 > gpurun_out/prof_w2v.log 2>&1 || exit 1
echo ALLDONE
