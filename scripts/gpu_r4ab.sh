#!/bin/bash
# Round 4: MF PS path identity plans on the local two-half layout (pair launch in delta mode).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4ab
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=300 step tests python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py tests/test_tensor_engine_gpu.py tests/test_vworld_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -k "tiled or mf or ps"
step mf_ps python -u bench.py --force-ps-path --no-hogwild-probe
step mf_ps2 python -u bench.py --force-ps-path --no-hogwild-probe
step local python -u bench.py --no-hogwild-probe
step prof rocprofv3 --kernel-trace --stats --output-format csv -d $O/mfps -o run -- python -u bench.py --force-ps-path --steps 6 --warmup 2 --no-hogwild-probe
echo ALLDONE
