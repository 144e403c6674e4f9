#!/bin/bash
# Round 4: Hogwild lost updates of the emulated N-GPU geometry with / without sub-step overlap; links at N = 2/4/8.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4u
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-600})"; }
step hog8_overlap python bench/probe_hogwild.py --users 1250000 --items 1000000 --per-user 51.2 --phases 1 --world 8
step hog8_serial python bench/probe_hogwild.py --users 1250000 --items 1000000 --per-user 51.2 --phases 1 --world 8 --overlap off
step hog2_overlap python bench/probe_hogwild.py --users 5000000 --items 1000000 --per-user 12.8 --phases 2 --world 2
step hog2_serial python bench/probe_hogwild.py --users 5000000 --items 1000000 --per-user 12.8 --phases 2 --world 2 --overlap off
W=2500 step links_overlap python -u bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3 --link-gbps 50
W=2500 step links_serial python -u bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3 --link-gbps 50 --overlap off
echo ALLDONE
