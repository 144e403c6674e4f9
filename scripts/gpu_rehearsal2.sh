#!/bin/bash
# Multi-rank rehearsal on one GPU (FPS_SHARE_GPU=1: every rank on cuda:0, gloo transport):
# the rotation + user-phase path of bench.py at N = 2 and 4, and the multi-rank GPU tests.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/reh2
for N in 2 4; do
  FPS_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2960$N bench.py --gpus $N --steps 3 --warmup 1 --batch 4194304 --user-phases 2 > gpurun_out/reh2/b_share$N.log 2>&1 || { tail -20 gpurun_out/reh2/b_share$N.log; exit 1; }
  echo "N=$N $(grep '^{' gpurun_out/reh2/b_share$N.log | cut -c1-160)"
done
timeout -k 10 400 python -u -m pytest tests/test_multirank_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/reh2/mr.log 2>&1 || { tail -20 gpurun_out/reh2/mr.log; exit 1; }
tail -1 gpurun_out/reh2/mr.log
echo ALLDONE
