#!/bin/bash
# Round 4: kernel trace of the local headline step (timeline vs the PS path's, gpurun_out/r4y).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4aa
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
step local rocprofv3 --kernel-trace --stats --output-format csv -d $O/local -o run -- python -u bench.py --steps 6 --warmup 2 --no-hogwild-probe
echo ALLDONE
