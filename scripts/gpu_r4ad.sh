#!/bin/bash
# Round 4: MF + top-K under the virtual world (candidate gather + PS through the runtime's communicator).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4ad
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -60 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=300 step tests python -u -m pytest tests/test_vworld_gpu.py tests/test_topk_tensor_gpu.py tests/test_topk_seen_merge_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread -k "mf_topk or topk or online"
echo ALLDONE
