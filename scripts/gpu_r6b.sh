#!/bin/bash
# Round 6: bench contract with the exact pass; collision-regime verify (world 1 on the GPU, 2 / 4 ranks sharing
# the GPU over gloo, store mutant); PA / SGNS PS paths on the hot-owner emulation (range / hash, zipf 0 / 1).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --verify > $O/bench_v.log 2>&1 || { tail -20 $O/bench_v.log; exit 1; }
tail -1 $O/bench_v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"],3), "%.4e" % d["value"], d["config"]["lost_user_update_fraction"], "exact", "%.4e" % d.get("exact_updates_per_s",0), d.get("exact_ms_per_step"), "verify", d["verify_ok"], {k: v for k, v in d["verify"].get("collision", {}).items() if "err" in k or "tol" in k or "lost" in k})'
timeout -k 10 120 python - > $O/collision_store.log 2>&1 <<'PY' || { tail -20 $O/collision_store.log; exit 1; }
import torch, json
from flink_parameter_server_1_amd.parallel.comm import Comm
from flink_parameter_server_1_amd.parallel.verify import rotation_check
c = Comm(device=torch.device("cuda", 0))
for uu in ("atomic", "store", "sc1"):
    r = rotation_check(c, user_update=uu, repeated_users=True)
    print(json.dumps({k: v for k, v in r.items() if k.startswith("verify_") and k != "verify_schedule"}))
PY
cat $O/collision_store.log
export FPS_SHARE_GPU=1
timeout -k 10 300 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 4194304 > $O/share2.log 2>&1 || { tail -30 $O/share2.log; exit 1; }
tail -1 $O/share2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("share2", d["config"]["user_update"], d["verify_ok"], "exact" in str(d.keys()), {k: v for k, v in d["verify"].get("collision", {}).items() if "err" in k or "tol" in k or "overlap" in k})'
timeout -k 10 300 python bench.py --gpus 4 --steps 3 --warmup 1 --batch 2097152 --users 2000000 > $O/share4.log 2>&1 || { tail -30 $O/share4.log; exit 1; }
tail -1 $O/share4.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("share4", d["config"]["user_update"], d["verify_ok"], {k: v for k, v in d["verify"].get("collision", {}).items() if "err" in k or "tol" in k or "overlap" in k})'
unset FPS_SHARE_GPU
for part in range hash; do
  for z in 1.0 0.0; do
    timeout -k 10 120 python bench/bench_pa.py --ps-path --steps 10 --warmup 3 --partition $part --zipf $z > $O/pa1_${part}_$z.log 2>&1 || { tail -20 $O/pa1_${part}_$z.log; exit 1; }
    echo "pa N=1 ps $part zipf=$z $(tail -1 $O/pa1_${part}_$z.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"])')"
    for n in 2 4 8; do
      timeout -k 10 120 python bench/bench_pa.py --emulate-world $n --steps 10 --warmup 3 --partition $part --zipf $z > $O/pa${n}_${part}_$z.log 2>&1 || { tail -20 $O/pa${n}_${part}_$z.log; exit 1; }
      echo "pa N=$n $part zipf=$z $(tail -1 $O/pa${n}_${part}_$z.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "rank", d["emulated_rank"], "shares", [round(x,3) for x in d["shard_key_shares"]], "wait", round(d["exposed_wait_ms_per_step"],3))')"
    done
  done
done
for n in 2 4 8; do
  timeout -k 10 120 python bench/bench_w2v.py --emulate-world $n --steps 10 --warmup 3 > $O/w2v${n}.log 2>&1 || { tail -20 $O/w2v${n}.log; exit 1; }
  echo "w2v N=$n $(tail -1 $O/w2v${n}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "rank", d["emulated_rank"], "wait", round(d["exposed_wait_ms_per_step"],3))')"
done
echo ALLDONE
