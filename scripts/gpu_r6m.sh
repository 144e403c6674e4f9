#!/bin/bash
# Round 6 (session 2): co-resident ("slim") partition kernels beside the tile SGD.
#  A = default build, fat partition;  B = default build, slim partition (SGD at 80 VGPRs: no room beside it)
#  C = SGD at <= 72 VGPRs (FPS_TG_MINW=7), fat;  D = SGD <= 72 VGPRs + slim partition (co-resident)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "tile_partition" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$PWD/flink_parameter_server_1_amd/_lib/ab/minw7/libfps_kernels.so
probe() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 180 python bench/probe_partition.py --steps 20 > $O/probe_$n.json 2> $O/probe_$n.err || { tail -20 $O/probe_$n.err; exit 1; }
  echo "$n $(cat $O/probe_$n.json)"
}
for r in 1 2; do
  probe A$r FPS_TP_SLIM=0
  probe B$r FPS_TP_SLIM=1
  probe C$r FPS_TP_SLIM=0 FPS_KERNELS_SO=$V
  probe D$r FPS_TP_SLIM=1 FPS_KERNELS_SO=$V
done
bench() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-hogwild-probe --exact-steps 0 > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
  echo "bench $n $(tail -1 $O/bench_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
}
bench A FPS_TP_SLIM=0
bench D FPS_TP_SLIM=1 FPS_KERNELS_SO=$V
bench A2 FPS_TP_SLIM=0
bench D2 FPS_TP_SLIM=1 FPS_KERNELS_SO=$V
FPS_TP_SLIM=1 FPS_KERNELS_SO=$V timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_D -- python bench/probe_partition.py --only step --steps 10 > $O/prof_D.log 2>&1 || { tail -20 $O/prof_D.log; exit 1; }
echo ALLDONE
