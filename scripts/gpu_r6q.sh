#!/bin/bash
# Round 6 (session 2): emulator receive fill as one kernel (segment_fill) -> PA / SGNS N = 8 re-measured;
# bf16 scorer stage size / query blocks A/B (LEMP + MF + top-K).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "segment_fill" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
run pa8_hash python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash
run pa8_range python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition range
run w2v8 python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
run w2v4 python bench/bench_w2v.py --emulate-world 4 --steps 10 --warmup 3
for r in 1 2; do
  for v in base st128 st256 qb1; do
    if [ $v = base ]; then S=""; else S=$PWD/flink_parameter_server_1_amd/_lib/ab/$v/libfps_kernels.so; fi
    run topk_${v}_$r env FPS_KERNELS_SO=$S python bench/bench_topk.py --steps 10 --warmup 3
    run mftopk_${v}_$r env FPS_KERNELS_SO=$S python bench/bench_mf_topk.py --steps 20 --warmup 3
  done
done
echo ALLDONE
