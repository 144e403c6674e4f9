#!/bin/bash
# Per-GPU compute of the N-GPU weak-scaling step, measured on one GPU: at N ranks each GPU
# holds 10M/N users and processes 64M ratings per step, so bench.py at N = 1 with
# --users 10M/N times the same SGD + partition work minus the ring transfers.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pergpu
for u in 10000000 5000000 2500000 1250000; do
  timeout -k 10 200 python bench.py --users $u --steps 20 --warmup 3 > gpurun_out/pergpu/u$u.log 2>&1 || { tail -20 gpurun_out/pergpu/u$u.log; exit 1; }
  echo "users=$u $(tail -1 gpurun_out/pergpu/u$u.log | cut -c1-170)"
done
