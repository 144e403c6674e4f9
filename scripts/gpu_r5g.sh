#!/bin/bash
# Round 5: same-box A/B of tile-SGD occupancy variants (rows in flight per lane group x workgroups per CU).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5g
mkdir -p $O
L=$PWD/flink_parameter_server_1_amd/_lib
for r in 1 2; do
  for v in base pf4 pf4w8 pf3 pf6 pf6w6; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-hogwild-probe > $O/ab_${v}_$r.log 2>&1 || { tail -20 $O/ab_${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 $O/ab_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
for v in base pf4w8; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  FPS_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-hogwild-probe --force-ps-path > $O/ps_${v}.log 2>&1 || { tail -20 $O/ps_${v}.log; exit 1; }
  FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 10 --warmup 3 > $O/emu8_${v}.log 2>&1 || { tail -20 $O/emu8_${v}.log; exit 1; }
  echo "$v ps $(tail -1 $O/ps_${v}.log | cut -c1-140) emu8 $(tail -1 $O/emu8_${v}.log | cut -c1-120)"
done
echo ALLDONE
