#!/bin/bash
# Round 3 final: full GPU validation (tests, smoke, headline bench + kernel stats) and the PA PS-path profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3z/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3z/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3z/smoke.log 2>&1 || { tail -20 gpurun_out/r3z/smoke.log; exit 1; }
tail -1 gpurun_out/r3z/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r3z/bench_n1.log 2>&1 || { tail -20 gpurun_out/r3z/bench_n1.log; exit 1; }
tail -1 gpurun_out/r3z/bench_n1.log | cut -c1-300
timeout -k 10 300 python bench/bench_pa.py --ps-path > gpurun_out/r3z/pa_ps.log 2>&1 || { tail -20 gpurun_out/r3z/pa_ps.log; exit 1; }
tail -1 gpurun_out/r3z/pa_ps.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3z/prof_pa -- python bench/bench_pa.py --ps-path --steps 5 --warmup 1 > gpurun_out/r3z/prof_pa.log 2>&1 || { tail -20 gpurun_out/r3z/prof_pa.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3z/prof_bench -- python bench.py --steps 5 --warmup 1 > gpurun_out/r3z/prof_bench.log 2>&1 || exit 1
echo ALLDONE
