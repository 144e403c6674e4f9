#!/bin/bash
# Flag dedup: numerics vs reference, PS-path benches (MF forced PS, SGNS PS path), kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/flg
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_tensor_ps_dist.py tests/test_multirank_gpu.py tests/test_kernels_grouped_gpu.py -m gpu -k "dedup or multirank or converge" -x -q --timeout 300 --timeout-method thread > gpurun_out/flg/tests.log 2>&1 || { tail -30 gpurun_out/flg/tests.log; exit 1; }
tail -1 gpurun_out/flg/tests.log
for M in flags; do
  FPS_DEDUP=$M timeout -k 10 300 python bench.py --force-ps-path --steps 10 --warmup 2 > gpurun_out/flg/mf_$M.log 2>&1 || { tail -20 gpurun_out/flg/mf_$M.log; exit 1; }
  echo "mf-ps $M $(grep '^{' gpurun_out/flg/mf_$M.log | cut -c80-190)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/flg/prof -- python bench.py --force-ps-path --steps 5 --warmup 1 > gpurun_out/flg/prof.log 2>&1 || exit 1
echo ALLDONE
