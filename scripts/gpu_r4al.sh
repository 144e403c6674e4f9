#!/bin/bash
# Round 4: partition side stream priority A/B (local headline and PS path).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4al
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-160})"; }
for rep in 1 2; do
  step local_norm_$rep python -u bench.py --no-hogwild-probe
  FPS_PART_PRIORITY=1 step local_high_$rep python -u bench.py --no-hogwild-probe
  step ps_norm_$rep python -u bench.py --force-ps-path --no-hogwild-probe
  FPS_PART_PRIORITY=1 step ps_high_$rep python -u bench.py --force-ps-path --no-hogwild-probe
done
echo ALLDONE
