#!/bin/bash
# Round 5: tile SGD with the chunk's records loaded once, all in flight (default) vs the count and placement
# passes each re-reading them one dependent load at a time (tg0 = HEAD) -- tests, then headline A/B.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5au
mkdir -p $O
L=flink_parameter_server_1_amd/_lib
timeout -k 10 400 python -u -m pytest tests/test_mf_tiled_gpu.py tests/test_kernels_gpu.py tests/test_hogwild_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
for r in 1 2 3; do
  for v in base tg0; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-hogwild-probe > $O/bench_${v}_$r.log 2>&1 || { tail -20 $O/bench_${v}_$r.log; exit 1; }
    echo "bench $v $r $(tail -1 $O/bench_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
for v in base tg0; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  FPS_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-hogwild-probe --force-ps-path > $O/ps_${v}.log 2>&1 || { tail -20 $O/ps_${v}.log; exit 1; }
  echo "ps $v $(tail -1 $O/ps_${v}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  FPS_KERNELS_SO=$so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-hogwild-probe --user-update atomic > $O/atomic_${v}.log 2>&1 || { tail -20 $O/atomic_${v}.log; exit 1; }
  echo "atomic $v $(tail -1 $O/atomic_${v}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
echo ALLDONE
