#!/bin/bash
# Round 4: MF PS path (presence from the partition, zero-copy identity serve), Hogwild counts (fixed least squares),
# bench JSON with the side probe, virtual world with a short GIL slice, emulated N = 8 kernel timeline.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4g
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-400})"; }
step tests python -u -m pytest tests/test_tensor_engine_gpu.py tests/test_mf_tiled_gpu.py tests/test_multirank_gpu.py tests/test_vworld_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
step probe_small python bench/probe_hogwild.py --users 1000000 --items 100000 --phases 4,1
step probe_store python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 4,1
step probe_sc1 python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 4 --user-update sc1
W=2000 step bench python bench.py
W=300 step mf_ps python bench.py --force-ps-path --steps 10 --no-hogwild-probe
step prof_mfps rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mfps -- python bench.py --force-ps-path --steps 5 --warmup 2 --no-hogwild-probe
for N in 2 4 8; do W=700 T=200 step vworld_n$N python -u bench/bench_vworld.py --world $N --traceback-s 60; done
T=400 step emulate8_trace rocprofv3 --kernel-trace --output-format csv -d $O/emu8 -- python bench/bench_emulate_world.py --ws 8 --steps 4 --warmup 2
echo ALLDONE
