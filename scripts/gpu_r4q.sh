#!/bin/bash
# Round 4: bf16 scorer (LENGTH variant) at 3 waves / SIMD (__launch_bounds__(256, 3), 168 VGPRs, 4 spilled) vs 2.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4q
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-200})"; }
step tests python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_seen_merge_gpu.py -m gpu -q --timeout 200 --timeout-method thread
for arm in lb3 lb2 lb3 lb2; do
  if [ $arm = lb2 ]; then export FPS_KERNELS_SO=$GRAFT_REPO_ROOT/ab/libfps_kernels_lb2.so; else unset FPS_KERNELS_SO; fi
  step topk_$arm python bench/bench_topk.py --strategy length
  step mftopk_$arm python bench/bench_mf_topk.py
done
echo ALLDONE
