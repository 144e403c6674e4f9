#!/bin/bash
# Round 4: three-digit radix threshold in topk_merge_kernel (seed segment merge).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4ag
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=300 step tests python -u -m pytest tests/test_topk_fast.py tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py tests/test_topk_seen_merge_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread
step topk python -u bench/bench_topk.py --strategy length
step mftopk python -u bench/bench_mf_topk.py
step mftopk2 python -u bench/bench_mf_topk.py
step prof rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench/bench_mf_topk.py --steps 8 --warmup 2
echo ALLDONE
