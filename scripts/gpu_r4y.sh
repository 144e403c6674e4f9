#!/bin/bash
# Round 4: kernel traces of the MF PS path (timeline gaps) and the fused SGNS PS path.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4y
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
step mfps rocprofv3 --kernel-trace --stats --output-format csv -d $O/mfps -o run -- python -u bench.py --force-ps-path --steps 6 --warmup 2 --no-hogwild-probe
step w2v rocprofv3 --kernel-trace --stats --output-format csv -d $O/w2v -o run -- python -u bench/bench_w2v.py --ps-path --steps 6 --warmup 2
step mfps_bench python -u bench.py --force-ps-path --no-hogwild-probe
echo ALLDONE
