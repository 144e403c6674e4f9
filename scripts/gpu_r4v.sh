#!/bin/bash
# Round 4: final rotation setting (overlap auto = from 4 ranks): virtual-world suite, emulated N with links, headline.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4v
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=400 step tests python -u -m pytest tests/test_vworld_gpu.py tests/test_multirank_gpu.py tests/test_mf_tiled_gpu.py tests/test_tensor_engine_gpu.py -m gpu -q --timeout 200 --timeout-method thread
W=2500 step links_auto python -u bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3 --link-gbps 50
W=2500 step links_auto2 python -u bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3 --link-gbps 50
W=2500 step nolinks_auto python -u bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3
W=1500 step bench python bench.py
echo ALLDONE
