#!/bin/bash
# Round 4: bf16 scorer reading per-block max lengths (scalar) -- 163 VGPRs, 3 waves / SIMD, no spills.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4r
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-200})"; }
step tests python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_seen_merge_gpu.py tests/test_topk_tensor.py tests/test_topk_fast.py -m gpu -q --timeout 200 --timeout-method thread
for st in length coord lc:1.3 length; do step topk_$st python bench/bench_topk.py --strategy $st; done
step mftopk1 python bench/bench_mf_topk.py
step mftopk2 python bench/bench_mf_topk.py
step prof_mftopk rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py --steps 6 --warmup 2
echo ALLDONE
