#!/bin/bash
# GPU: prefetch A/B on one box at the default tile policy; clean per-kernel profile without prefetch.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 > gpurun_out/b_pf$i.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --steps 20 --no-prefetch > gpurun_out/b_nopf$i.log 2>&1 || exit 1
  echo "prefetch: $(tail -1 gpurun_out/b_pf$i.log | cut -c60-120)   no-prefetch: $(tail -1 gpurun_out/b_nopf$i.log | cut -c60-120)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/nopf -- python bench.py --steps 5 --warmup 1 --no-prefetch > gpurun_out/prof_nopf.log 2>&1 || exit 1
echo ALLDONE
