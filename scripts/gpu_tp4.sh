#!/bin/bash
# tp4 (capacity-slot partition): prefetch/sync probe, same-box A/B vs tp3, kernel stats.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tp4
timeout -k 10 300 python -u scripts/probe_prefetch.py > gpurun_out/tp4/probe.log 2>&1 || { tail -20 gpurun_out/tp4/probe.log; exit 1; }
cat gpurun_out/tp4/probe.log | grep levels
for rep in 1 2; do
  for lv in 3 4; do
    FPS_TILE_PARTITION_LEVELS=$lv timeout -k 10 200 python bench.py > gpurun_out/tp4/bench_L${lv}_$rep.log 2>&1 || { tail -20 gpurun_out/tp4/bench_L${lv}_$rep.log; exit 1; }
    echo "L$lv rep$rep $(tail -1 gpurun_out/tp4/bench_L${lv}_$rep.log | cut -c1-190)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp4/prof_nopf -- python bench.py --steps 5 --warmup 2 --no-prefetch > gpurun_out/tp4/prof_nopf.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp4/prof_pf -- python bench.py --steps 5 --warmup 2 > gpurun_out/tp4/prof_pf.log 2>&1 || exit 1
echo ALLDONE
