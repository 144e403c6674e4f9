#!/bin/bash
# Round 5: same-box A/B of tile-SGD build variants (user rows in flight per lane group, occupancy), and the
# secondary PS paths (PA, SGNS) at N = 1 / 2 / 4 / 8 under the rank-symmetric emulation (parallel/emulated.py).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5d
mkdir -p $O
L=flink_parameter_server_1_amd/_lib
for r in 1 2; do
  for v in base pf10 pf4 minw6; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$PWD/$so timeout -k 10 300 python bench.py --steps 15 --warmup 3 --no-hogwild-probe > $O/ab_${v}_$r.log 2>&1 || { tail -20 $O/ab_${v}_$r.log; exit 1; }
    echo "$v $r $(tail -1 $O/ab_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
for N in 1 2 4 8; do
  em=""; [ $N -gt 1 ] && em="--emulate-world $N --link-gbps 50"
  timeout -k 10 300 python bench/bench_pa.py --ps-path $em > $O/pa_$N.log 2>&1 || { tail -20 $O/pa_$N.log; exit 1; }
  tail -1 $O/pa_$N.log | cut -c1-160
  timeout -k 10 300 python bench/bench_w2v.py --ps-path $em > $O/w2v_$N.log 2>&1 || { tail -20 $O/w2v_$N.log; exit 1; }
  tail -1 $O/w2v_$N.log | cut -c1-160
done
for N in 8; do
  timeout -k 10 300 python bench/bench_pa.py --ps-path --emulate-world $N --link-gbps 50 --wire bf16 > $O/pa_${N}_bf16.log 2>&1 || { tail -20 $O/pa_${N}_bf16.log; exit 1; }
  timeout -k 10 300 python bench/bench_w2v.py --ps-path --emulate-world $N --link-gbps 50 --wire bf16 > $O/w2v_${N}_bf16.log 2>&1 || { tail -20 $O/w2v_${N}_bf16.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --ps-path --emulate-world 8 --steps 6 --warmup 2 > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2v8 -- python bench/bench_w2v.py --ps-path --emulate-world 8 --steps 6 --warmup 2 > $O/prof_w2v8.log 2>&1 || { tail -20 $O/prof_w2v8.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_hogwild_gpu.py -x -v --timeout 500 --timeout-method thread > $O/hogwild.log 2>&1 || { tail -40 $O/hogwild.log; exit 1; }
grep -E "PASS|FAIL" $O/hogwild.log
for uu in atomic store; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 --user-update $uu > $O/bench_$uu.log 2>&1 || { tail -20 $O/bench_$uu.log; exit 1; }
  tail -1 $O/bench_$uu.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["user_update"], round(d["ms_per_step"],3), "%.4e" % d["value"], d["config"]["lost_user_update_fraction"], d["effective_updates_per_s"])'
  timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 10 --warmup 3 --user-update $uu > $O/emu8_$uu.log 2>&1 || { tail -20 $O/emu8_$uu.log; exit 1; }
  tail -1 $O/emu8_$uu.log | cut -c1-300
done
echo ALLDONE
