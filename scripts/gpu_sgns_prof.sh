#!/bin/bash
# SGNS round-2 kernel: GPU tests (kernel + model + multi-rank rehearsal), bench, kernel profile
set -e
mkdir -p gpurun_out/sgns
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sgns_sampling.py tests/test_multirank_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sgns/tests2.log 2>&1 || { tail -30 gpurun_out/sgns/tests2.log; exit 1; }
tail -1 gpurun_out/sgns/tests2.log
timeout -k 10 200 python bench/bench_w2v.py > gpurun_out/sgns/w2v_default.json && tail -1 gpurun_out/sgns/w2v_default.json | cut -c1-300
timeout -k 10 200 python bench/bench_w2v.py --ps-path > gpurun_out/sgns/w2v_ps.json && tail -1 gpurun_out/sgns/w2v_ps.json | cut -c1-200
rm -rf gpurun_out/sgns/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sgns/prof -- python bench/bench_w2v.py --steps 10 > gpurun_out/sgns/prof.log 2>&1 || { tail -20 gpurun_out/sgns/prof.log; exit 1; }
