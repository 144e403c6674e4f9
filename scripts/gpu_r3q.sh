#!/bin/bash
# Round 3: tile rows at the emulated N = 4 / 8 rotation step (per-GPU compute), same box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3q
for rep in 1 2; do
  for R in auto 32 64 128; do
    if [ $R = auto ]; then unset FPS_TILE_ROWS; else export FPS_TILE_ROWS=$R; fi
    timeout -k 10 400 python bench/bench_emulate_world.py --ws 4,8 > gpurun_out/r3q/emu_$R.$rep.log 2>&1 || { tail -20 gpurun_out/r3q/emu_$R.$rep.log; exit 1; }
    echo "R=$R rep $rep"; grep -o '"emulated_world": [0-9]*\|"ms_per_step": [0-9.]*\|"tile_rows": [0-9]*' gpurun_out/r3q/emu_$R.$rep.log | paste -sd' '
  done
done
unset FPS_TILE_ROWS
echo ALLDONE
