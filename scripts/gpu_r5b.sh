#!/bin/bash
# Round 5: sentinel race tests, smoke, per-user atomics probe, headline bench + kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5b
timeout -k 10 300 python -u -m pytest tests/test_touch_sentinel.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5b/tests.log 2>&1 || { tail -30 gpurun_out/r5b/tests.log; exit 1; }
tail -2 gpurun_out/r5b/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5b/smoke.log 2>&1 || { tail -20 gpurun_out/r5b/smoke.log; exit 1; }
tail -1 gpurun_out/r5b/smoke.log
timeout -k 10 300 python -u bench/probe_atomics.py > gpurun_out/r5b/atomics.jsonl 2>&1 || { tail -20 gpurun_out/r5b/atomics.jsonl; exit 1; }
cat gpurun_out/r5b/atomics.jsonl
timeout -k 10 300 python bench.py > gpurun_out/r5b/bench_n1.log 2>&1 || { tail -20 gpurun_out/r5b/bench_n1.log; exit 1; }
tail -1 gpurun_out/r5b/bench_n1.log | cut -c1-400
echo ALLDONE
