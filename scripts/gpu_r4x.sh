#!/bin/bash
# Round 4: SGNS PS path with the world-1 push fused into the kernel (write maps), A/B against pushed deltas.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4x
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-400})"; }
T=300 step tests python -u -m pytest tests/test_sgns_sampling.py tests/test_vworld_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -k "sgns"
step ps_fused python -u bench/bench_w2v.py --ps-path
step ps_unfused python -u bench/bench_w2v.py --ps-path --no-fuse-local-push
step ps_fused2 python -u bench/bench_w2v.py --ps-path
step direct python -u bench/bench_w2v.py
T=300 step prof rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u bench/bench_w2v.py --ps-path --steps 8 --warmup 2
echo ALLDONE
