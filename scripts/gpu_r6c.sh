#!/bin/bash
# Round 6: kernel profiles of the emulated N = 8 PA (hash, fp64 feature draws) and SGNS PS paths; bench --verify with the
# fixed collision criterion.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --verify > $O/bench_v.log 2>&1 || { tail -20 $O/bench_v.log; exit 1; }
tail -1 $O/bench_v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"],3), "%.4e" % d["value"], d["config"]["lost_user_update_fraction"], "exact", "%.4e" % d.get("exact_updates_per_s",0), d.get("exact_ms_per_step"), "verify", d["verify_ok"], {k: v for k, v in d["verify"].get("collision", {}).items() if "err" in k or "tol" in k or "ok" in k})'
for part in hash range; do
  timeout -k 10 120 python bench/bench_pa.py --emulate-world 8 --steps 10 --warmup 3 --partition $part > $O/pa8_$part.log 2>&1 || { tail -20 $O/pa8_$part.log; exit 1; }
  echo "pa N=8 $part $(tail -1 $O/pa8_$part.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "rank", d["emulated_rank"], "shares", [round(x,3) for x in d["shard_key_shares"]], "wait", round(d["exposed_wait_ms_per_step"],3))')"
done
timeout -k 10 120 python bench/bench_pa.py --ps-path --steps 10 --warmup 3 --partition hash > $O/pa1_hash.log 2>&1 || { tail -20 $O/pa1_hash.log; exit 1; }
echo "pa N=1 ps hash $(tail -1 $O/pa1_hash.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"])')"
timeout -k 10 120 python bench/bench_pa.py --ps-path --no-fuse-local-push --steps 10 --warmup 3 --partition hash > $O/pa1_hash_nf.log 2>&1 || { tail -20 $O/pa1_hash_nf.log; exit 1; }
echo "pa N=1 ps hash delta-buffer $(tail -1 $O/pa1_hash_nf.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"])')"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --emulate-world 8 --steps 10 --warmup 3 --partition hash > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2v8 -- python bench/bench_w2v.py --emulate-world 8 --steps 6 --warmup 2 > $O/prof_w2v8.log 2>&1 || { tail -20 $O/prof_w2v8.log; exit 1; }
echo ALLDONE
