#!/bin/bash
# Round 5: pipelined loads in dedup assign/resolve, hash-table assign, top-k merge -- same-box A/B against the
# kernels one commit earlier ("preload" variant), alternating: MF + top-K, PA PS path emulated at N = 8, capacity.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5r
mkdir -p $O
L=$PWD/flink_parameter_server_1_amd/_lib
for r in 1 2; do
  for v in base preload; do
    so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "mftopk $v $r $(tail -1 $O/mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
    FPS_KERNELS_SO=$so timeout -k 10 300 python bench/bench_pa.py --ps-path --emulate-world 8 > $O/pa8_${v}_$r.log 2>&1 || { tail -20 $O/pa8_${v}_$r.log; exit 1; }
    echo "pa8 $v $r $(tail -1 $O/pa8_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["per_gpu_rate"])')"
  done
done
for v in base preload; do
  so=$L/libfps_kernels.so; [ $v != base ] && so=$L/ab/$v/libfps_kernels.so
  FPS_KERNELS_SO=$so timeout -k 10 400 python bench/bench_capacity.py > $O/cap_$v.log 2>&1 || { tail -20 $O/cap_$v.log; exit 1; }
  echo "capacity $v $(tail -1 $O/cap_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
echo ALLDONE
