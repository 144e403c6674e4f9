#!/bin/bash
# Round 4: persistent tiled SGD A/B (N = 1 headline, emulated N = 8), vworld control runs without link delay.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4i
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
step tests python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py -m gpu -x -q -k "tiled or persistent" --timeout 200 --timeout-method thread
for i in 1 2; do
  W=200 step bench_plain_$i python bench.py --no-hogwild-probe
  W=200 step bench_pers_$i python bench.py --no-hogwild-probe --persistent-sgd
done
T=400 step emu python bench/bench_emulate_world.py --ws 1,8 --steps 10 --warmup 3
T=400 step emu_pers python bench/bench_emulate_world.py --ws 1,8 --steps 10 --warmup 3 --persistent-sgd
W=200 step mfps_pers python bench.py --force-ps-path --steps 10 --no-hogwild-probe --persistent-sgd
for N in 4 8; do W=700 T=200 step vworld_nodelay_n$N python -u bench/bench_vworld.py --world $N --no-delay --traceback-s 60; done
echo ALLDONE
