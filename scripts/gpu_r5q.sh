#!/bin/bash
# Round 5: SGNS shared-negative MFMA kernel with unconditional staging loads -- numerics, then a same-box A/B vs the
# guarded loads (variant "guarded"), in place and through the PS path.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5q
mkdir -p $O
L=$PWD/flink_parameter_server_1_amd/_lib
timeout -k 10 600 python -u -m pytest -m gpu tests/test_sgns_sampling.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in base guarded; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_w2v.py --mode shared > $O/shared_${v}_$r.log 2>&1 || { tail -20 $O/shared_${v}_$r.log; exit 1; }
    echo "shared $v $r $(tail -1 $O/shared_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
for v in base guarded; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_w2v.py --mode shared --ps-path > $O/shared_ps_$v.log 2>&1 || { tail -20 $O/shared_ps_$v.log; exit 1; }
  echo "shared-ps $v $(tail -1 $O/shared_ps_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
echo ALLDONE
