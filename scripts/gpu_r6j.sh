#!/bin/bash
# Round 6: config #5 at N = 8 on the hot-owner emulation (12.5e9-parameter shard, Adagrad, staleness 2), owner stream
# vs interleaved; SGNS emulated after the revert.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sgns_sampling.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
runc() {
  local n=$1; shift
  timeout -k 10 300 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["value"], "pairs/s %.3e" % d["pairs_per_s"], "wait", d.get("exposed_wait_ms_per_step"), "hbm", round(d["peak_hbm_gib_rank0"],1), "rank", d.get("emulated_rank"), d["config"].get("owner_stream"), d["config"].get("interleaved"), "loss", round(d["eval_loss_before"],3), round(d["eval_loss_after"],3))')"
}
runc cap1 python bench/bench_capacity.py --steps 20 --warmup 3
runc cap8 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8
FPS_OWNER_STREAM=0 runc cap8_noowner python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 150 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", d["exposed_wait_ms_per_step"] and round(d["exposed_wait_ms_per_step"],3))')"
}
for n in 2 4 8; do
  run w2v$n python bench/bench_w2v.py --emulate-world $n --steps 10 --warmup 3
done
FPS_OWNER_STREAM=0 run w2v8_noowner python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
echo ALLDONE
