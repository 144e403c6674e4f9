#!/bin/bash
# Full GPU validation on one MI355X: gpu test suite, smoke(), headline bench (N = 1 and the N = 2 rehearsal on one
# GPU), kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/validate
mkdir -p $O/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc" >> $O/gpu_tests.log
tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_n1.log 2>&1 || { tail -20 $O/bench_n1.log; exit 1; }
tail -1 $O/bench_n1.log | cut -c1-300
FPS_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 4194304 > $O/bench_n2.log 2>&1 || { tail -30 $O/bench_n2.log; exit 1; }
grep '^{' $O/bench_n2.log | cut -c1-300
FPS_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 3 --warmup 1 --batch 2097152 > $O/bench_n4.log 2>&1 || { tail -30 $O/bench_n4.log; exit 1; }
grep '^{' $O/bench_n4.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof/bench -- python bench.py --steps 5 --warmup 1 > $O/prof_bench.log 2>&1 || exit 1
echo ALLDONE
