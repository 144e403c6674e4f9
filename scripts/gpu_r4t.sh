#!/bin/bash
# Round 4: rotation sub-steps on alternating compute streams -- virtual-world correctness, emulated N A/B.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4t
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=400 step tests python -u -m pytest tests/test_vworld_gpu.py tests/test_multirank_gpu.py tests/test_mf_tiled_gpu.py -m gpu -q --timeout 200 --timeout-method thread
W=2500 T=400 step emu_overlap python -u bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3
W=2500 T=400 step emu_serial python -u bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3 --overlap off
W=2500 T=400 step emu_overlap_links python -u bench/bench_emulate_world.py --ws 8 --steps 10 --warmup 3 --link-gbps 50
W=2500 T=400 step emu_overlap2 python -u bench/bench_emulate_world.py --ws 1,8 --steps 10 --warmup 3
W=2500 T=400 step emu_serial2 python -u bench/bench_emulate_world.py --ws 1,8 --steps 10 --warmup 3 --overlap off
T=400 step emu8_trace rocprofv3 --kernel-trace --output-format csv -d $O/emu8 -- python bench/bench_emulate_world.py --ws 8 --steps 4 --warmup 2
echo ALLDONE
