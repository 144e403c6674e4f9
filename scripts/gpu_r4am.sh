#!/bin/bash
# Round 4 end: LEMP strategies after the seed-merge change (COORD / LC vs LENGTH).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4am
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-140})"; }
for rep in 1 2; do
  step length_$rep python -u bench/bench_topk.py --strategy length
  step coord_$rep python -u bench/bench_topk.py --strategy coord
  step lc_$rep python -u bench/bench_topk.py --strategy lc:1.3
done
echo ALLDONE
