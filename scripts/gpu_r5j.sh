#!/bin/bash
# Round 5: count kernel with non-returning LDS atomics (FPS_TP_NORET=1) -- partition tests on the variant, then a
# same-box A/B of the headline and the N = 8 emulated step (alternating).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5j
mkdir -p $O
L=$PWD/flink_parameter_server_1_amd/_lib
FPS_KERNELS_SO=$L/ab/noret/libfps_kernels.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "tile_partition" -x -q --timeout 300 --timeout-method thread > $O/tests_noret.log 2>&1 || { tail -40 $O/tests_noret.log; exit 1; }
tail -1 $O/tests_noret.log
for r in 1 2; do
  for v in base noret; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-hogwild-probe > $O/ab_${v}_$r.log 2>&1 || { tail -20 $O/ab_${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 $O/ab_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
for v in base noret; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 10 --warmup 3 > $O/emu8_${v}.log 2>&1 || { tail -20 $O/emu8_${v}.log; exit 1; }
  echo "$v emu8 $(tail -1 $O/emu8_${v}.log | cut -c1-120)"
done
FPS_KERNELS_SO=$L/ab/noret/libfps_kernels.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_noret -- python bench.py --steps 5 --warmup 2 --no-hogwild-probe > $O/prof_noret.log 2>&1 || { tail -20 $O/prof_noret.log; exit 1; }
echo ALLDONE
