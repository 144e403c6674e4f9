#!/bin/bash
# Round 6 session 3, closing numbers on the final build: headline x2, emulated MF rotation (fresh process per N, 50 GB/s
# links), PA / SGNS at N = 8 on the hot-owner emulation, LEMP top-K and MF + top-K.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3final2
mkdir -p $O
for r in 1 2; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
  tail -1 $O/bench_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"],3), "%.4e" % d["value"], "lost", round(d["config"]["lost_user_update_fraction"],4), "eff %.4e" % d["effective_updates_per_s"], "exact %.4e" % d.get("exact_updates_per_s",0), round(d.get("exact_ms_per_step", 0), 3))'
done
timeout -k 10 300 python bench/bench_emulate_world.py --ws 2,4,8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu_links.jsonl 2>$O/emu_links.err || { tail -20 $O/emu_links.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r6s3final2/emu_links.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print("emu_links", d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], d["user_update"], round(d["comm_wait_ms_per_step"], 3))
PY
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
run pa8_hash python bench/bench_pa.py --emulate-world 8 --steps 80 --warmup 5 --partition hash
run pa8_range python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition range
run w2v8 python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3
timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk.log 2>&1 || { tail -20 $O/topk.log; exit 1; }
echo "topk $(tail -1 $O/topk.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk.log 2>&1 || { tail -20 $O/mftopk.log; exit 1; }
echo "mftopk $(tail -1 $O/mftopk.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
echo ALLDONE
