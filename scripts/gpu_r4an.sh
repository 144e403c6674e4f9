#!/bin/bash
# Round 4: bf16 scorer query blocks per wave (QB = 4 default vs 2) A/B on LEMP and MF + top-K.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4an
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-140})"; }
FPS_SB_QB=2 T=300 step tests python -u -m pytest tests/test_topk_bf16_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread
for rep in 1 2; do
  step topk_qb4_$rep python -u bench/bench_topk.py --strategy length
  FPS_SB_QB=2 step topk_qb2_$rep python -u bench/bench_topk.py --strategy length
  step mftopk_qb4_$rep python -u bench/bench_mf_topk.py
  FPS_SB_QB=2 step mftopk_qb2_$rep python -u bench/bench_mf_topk.py
done
echo ALLDONE
