#!/bin/bash
# Rehearse the driver's N>1 bench launch on one GPU (ranks share cuda:0, gloo host-staged transport).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for N in 2 4; do
  FPS_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2950$N bench.py --gpus $N --steps 3 --warmup 1 --batch 4194304 > gpurun_out/b_share$N.log 2>&1 || exit 1
  grep metric gpurun_out/b_share$N.log | cut -c1-250
done
FPS_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --batch 4194304 --exchange ps > gpurun_out/b_share2ps.log 2>&1 || exit 1
grep metric gpurun_out/b_share2ps.log | cut -c1-250
echo ALLDONE
