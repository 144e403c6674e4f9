#!/bin/bash
# Round 4: PA PS path with the world-1 push applied by the PA kernel (write map), A/B.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4ac
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=300 step tests python -u -m pytest tests/test_pa_fast.py tests/test_pa_offline_tensor_gpu.py tests/test_touch_sentinel.py tests/test_vworld_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread
step pa_fused python -u bench/bench_pa.py --ps-path
step pa_unfused python -u bench/bench_pa.py --ps-path --no-fuse-local-push
step pa_fused2 python -u bench/bench_pa.py --ps-path
step pa_direct python -u bench/bench_pa.py
step prof rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench/bench_pa.py --ps-path --steps 8 --warmup 2
echo ALLDONE
