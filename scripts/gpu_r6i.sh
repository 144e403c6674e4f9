#!/bin/bash
# Round 6: SGNS bf16-row kernels: tests, emulated N = 2/4/8, N = 1 PS paths.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sgns_sampling.py tests/test_multigpu_nccl_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 150 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", d["exposed_wait_ms_per_step"] and round(d["exposed_wait_ms_per_step"],3), "loss", d["loss_first_last"])')"
}
run w2v1_direct python bench/bench_w2v.py --steps 10 --warmup 3
run w2v1_ps python bench/bench_w2v.py --steps 10 --warmup 3 --ps-path
run w2v1_ps_bf16 python bench/bench_w2v.py --steps 10 --warmup 3 --ps-path --wire bf16 --no-fuse-local-push
for n in 2 4 8; do
  run w2v$n python bench/bench_w2v.py --emulate-world $n --steps 10 --warmup 3
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2v8 -- python bench/bench_w2v.py --emulate-world 8 --steps 6 --warmup 2 > $O/prof_w2v8.log 2>&1 || { tail -20 $O/prof_w2v8.log; exit 1; }
echo ALLDONE
