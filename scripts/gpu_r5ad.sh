#!/bin/bash
# Round 5: presence marked by the level-2 scatter ('base') vs by the count pass ('cntseen', one commit earlier) --
# partition tests, then MF PS path and the emulated N = 8 rotation (exact and Hogwild), alternating.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ad
mkdir -p $O
L=$PWD/flink_parameter_server_1_amd/_lib
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "tile_partition" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u -m pytest tests/test_tensor_engine_gpu.py tests/test_vworld_gpu.py -k "mf" -x -q --timeout 300 --timeout-method thread > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
for r in 1 2; do
  for v in base cntseen; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --force-ps-path --no-hogwild-probe > $O/ps_${v}_$r.log 2>&1 || { tail -20 $O/ps_${v}_$r.log; exit 1; }
    echo "ps $v $r $(tail -1 $O/ps_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 8 --warmup 2 > $O/emu8_${v}_$r.log 2>&1 || { tail -20 $O/emu8_${v}_$r.log; exit 1; }
    echo "emu8-exact $v $r $(tail -1 $O/emu8_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["updates_per_s_per_gpu"])')"
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 8 --warmup 2 --user-update store > $O/emu8s_${v}_$r.log 2>&1 || { tail -20 $O/emu8s_${v}_$r.log; exit 1; }
    echo "emu8-store $v $r $(tail -1 $O/emu8s_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["updates_per_s_per_gpu"])')"
  done
done
echo ALLDONE
