#!/bin/bash
# Round 4: MF PS path vs user phases (partition interference / launch tails).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4af
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-200})"; }
for P in 2 3 4 5 6 8; do
  step ps_p$P python -u bench.py --force-ps-path --no-hogwild-probe --user-phases $P
done
echo ALLDONE
