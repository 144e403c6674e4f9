#!/bin/bash
# Round 4: bf16 scorer with MFMA accumulators in VGPRs (-amdgpu-mfma-vgpr-form) vs the AGPR form, same box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4p
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-200})"; }
step tests python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_seen_merge_gpu.py tests/test_topk_fast.py -m gpu -q --timeout 200 --timeout-method thread
for arm in vgpr agpr vgpr agpr; do
  if [ $arm = agpr ]; then export FPS_KERNELS_SO=$GRAFT_REPO_ROOT/ab/libfps_kernels_agpr.so; else unset FPS_KERNELS_SO; fi
  step topk_$arm python bench/bench_topk.py --strategy length
  step mftopk_$arm python bench/bench_mf_topk.py
done
unset FPS_KERNELS_SO
step prof_topk rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_topk -- python bench/bench_topk.py --strategy length --steps 5 --warmup 1
echo ALLDONE
