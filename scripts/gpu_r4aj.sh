#!/bin/bash
# Round 4: local headline vs user phases with 16-bit count counters everywhere.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4aj
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-160})"; }
for rep in 1 2; do
  for P in 3 4 5 6; do
    step local_p${P}_$rep python -u bench.py --no-hogwild-probe --user-phases $P
  done
done
echo ALLDONE
