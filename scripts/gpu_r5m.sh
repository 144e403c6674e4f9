#!/bin/bash
# Round 5: partition grid cap (FPS_TP_GRID: fewer, looping partition workgroups beside the SGD) -- tests with a small
# cap, then a same-box A/B of the headline (alternating); MF PS path after the stats change.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5m
mkdir -p $O
FPS_TP_GRID=24 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "tile_partition" -x -q --timeout 300 --timeout-method thread > $O/tests_grid.log 2>&1 || { tail -40 $O/tests_grid.log; exit 1; }
tail -1 $O/tests_grid.log
for r in 1 2; do
  for g in 0 64 128 256; do
    FPS_TP_GRID=$g timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-hogwild-probe > $O/ab_${g}_$r.log 2>&1 || { tail -20 $O/ab_${g}_$r.log; exit 1; }
    echo "grid $g $r $(tail -1 $O/ab_${g}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --force-ps-path --no-hogwild-probe > $O/ps_$r.log 2>&1 || { tail -20 $O/ps_$r.log; exit 1; }
  echo "ps $r $(tail -1 $O/ps_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
echo ALLDONE
