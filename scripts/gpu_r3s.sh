#!/bin/bash
# Round 3: count-kernel workgroups when its histogram exceeds 64 KiB of LDS (emulated N = 8 / 4 step and N = 1),
# 512 (tree default) vs 128 vs 64 (_lib/ab builds), same box, alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3s
AB=$GRAFT_REPO_ROOT/flink_parameter_server_1_amd/_lib/ab
for rep in 1 2; do
  for v in 512 128 64; do
    if [ $v = 512 ]; then unset FPS_KERNELS_SO; else export FPS_KERNELS_SO=$AB/libfps_kernels_$v.so; fi
    timeout -k 10 400 python bench/bench_emulate_world.py --ws 8,4,1 > gpurun_out/r3s/emu_$v.$rep.log 2>&1 || { tail -20 gpurun_out/r3s/emu_$v.$rep.log; exit 1; }
    echo "cap=$v rep $rep $(grep -o '"emulated_world": [0-9]*\|"ms_per_step": [0-9.]*' gpurun_out/r3s/emu_$v.$rep.log | paste -sd' ')"
  done
done
unset FPS_KERNELS_SO
echo ALLDONE
