#!/bin/bash
# PS-protocol cost on one MI355X: PA and MF through the tensor engine (pull / push) vs in place,
# engine plumbing per micro-batch, kernel stats of the PS paths.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3d
timeout -k 10 300 python bench/bench_pa.py --ps-path > gpurun_out/r3d/pa_ps.log 2>&1 || { tail -20 gpurun_out/r3d/pa_ps.log; exit 1; }
tail -1 gpurun_out/r3d/pa_ps.log | cut -c1-160
timeout -k 10 300 python bench/bench_pa.py > gpurun_out/r3d/pa_direct.log 2>&1 || { tail -20 gpurun_out/r3d/pa_direct.log; exit 1; }
tail -1 gpurun_out/r3d/pa_direct.log | cut -c1-160
timeout -k 10 300 python bench.py --force-ps-path --steps 10 > gpurun_out/r3d/mf_ps.log 2>&1 || { tail -20 gpurun_out/r3d/mf_ps.log; exit 1; }
tail -1 gpurun_out/r3d/mf_ps.log | cut -c1-160
timeout -k 10 300 python bench/bench_engine.py --batches 1,64,4096,262144 > gpurun_out/r3d/engine.log 2>&1 || { tail -20 gpurun_out/r3d/engine.log; exit 1; }
tail -1 gpurun_out/r3d/engine.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d/prof_pa -- python bench/bench_pa.py --ps-path --steps 5 --warmup 1 > gpurun_out/r3d/prof_pa.log 2>&1 || { tail -20 gpurun_out/r3d/prof_pa.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d/prof_mfps -- python bench.py --force-ps-path --steps 5 --warmup 1 > gpurun_out/r3d/prof_mfps.log 2>&1 || { tail -20 gpurun_out/r3d/prof_mfps.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d/prof_w2v -- python bench/bench_w2v.py --steps 5 --warmup 1 > gpurun_out/r3d/prof_w2v.log 2>&1 || { tail -20 gpurun_out/r3d/prof_w2v.log; exit 1; }
find gpurun_out/r3d -name "*kernel_stats.csv" | head
echo ALLDONE
