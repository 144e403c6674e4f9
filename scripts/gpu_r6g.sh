#!/bin/bash
# Round 6: PA PS path vs batch size (host overhead per micro-batch) at N = 1 / 8 (hash, range).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g
mkdir -p $O
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 120 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d["per_gpu_rate"], "wait", d["exposed_wait_ms_per_step"] and round(d["exposed_wait_ms_per_step"],3))')"
}
for b in 65536 262144; do
  run pa1_ps_b$b python bench/bench_pa.py --ps-path --steps 20 --warmup 3 --partition hash --batch $b
  run pa1_ps_nofuse_b$b python bench/bench_pa.py --ps-path --no-fuse-local-push --steps 20 --warmup 3 --partition hash --batch $b
  run pa1_direct_b$b python bench/bench_pa.py --steps 20 --warmup 3 --partition hash --batch $b
  run pa8_hash_b$b python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition hash --batch $b
  run pa8_range_b$b python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition range --batch $b
  run pa4_hash_b$b python bench/bench_pa.py --emulate-world 4 --steps 20 --warmup 3 --partition hash --batch $b
  run pa2_hash_b$b python bench/bench_pa.py --emulate-world 2 --steps 20 --warmup 3 --partition hash --batch $b
done
echo ALLDONE
