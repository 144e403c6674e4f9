#!/bin/bash
# Round 6 final measurements (session 2, after the PS-path trims and the unrolled link fill): headline x2 (+ exact rate), timed-loop kernel profile, emulated MF rotation scaling,
# PA / SGNS / config #5 PS paths on the hot-owner emulation, N = 1 PS paths.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6final3
mkdir -p $O
for r in 1 2; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
  tail -1 $O/bench_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"],3), "%.4e" % d["value"], "lost", round(d["config"]["lost_user_update_fraction"],4), "eff %.4e" % d["effective_updates_per_s"], "exact %.4e" % d.get("exact_updates_per_s",0), round(d.get("exact_ms_per_step", 0), 3))'
done
timeout -k 10 300 python bench/bench_emulate_world.py --ws 1,2,4,8 --steps 20 --warmup 5 > $O/emu.jsonl 2>$O/emu.err || { tail -20 $O/emu.err; exit 1; }
timeout -k 10 300 python bench/bench_emulate_world.py --ws 2,4,8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu_links.jsonl 2>$O/emu_links.err || { tail -20 $O/emu_links.err; exit 1; }
python - <<'PY'
import json
for f in ("emu", "emu_links"):
    for l in open(f"gpurun_out/r6final3/{f}.jsonl"):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], d["user_update"], round(d["comm_wait_ms_per_step"], 3))
PY
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.3e" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
run pa1_direct python bench/bench_pa.py --steps 20 --warmup 3 --partition hash
run pa1_ps python bench/bench_pa.py --ps-path --steps 20 --warmup 3 --partition hash
run pa1_ps_delta python bench/bench_pa.py --ps-path --no-fuse-local-push --steps 20 --warmup 3 --partition hash
for n in 2 4 8; do
  run pa${n}_hash python bench/bench_pa.py --emulate-world $n --steps 80 --warmup 5 --partition hash
  run pa${n}_range python bench/bench_pa.py --emulate-world $n --steps 20 --warmup 3 --partition range
done
run pa8_hash_z0 python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition hash --zipf 0
run pa8_range_z0 python bench/bench_pa.py --emulate-world 8 --steps 20 --warmup 3 --partition range --zipf 0
run w2v1_direct python bench/bench_w2v.py --steps 10 --warmup 3
run w2v1_ps python bench/bench_w2v.py --steps 10 --warmup 3 --ps-path
for n in 2 4 8; do
  run w2v$n python bench/bench_w2v.py --emulate-world $n --steps 10 --warmup 3
done
run cap1 python bench/bench_capacity.py --steps 20 --warmup 3
run cap8 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8
run cap8_bf16 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8 --wire bf16
run w2v1_ps_bf16 python bench/bench_w2v.py --steps 10 --warmup 3 --ps-path --wire bf16
run pa8_hash_b python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash
run pa8_hash_dedup python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash --dedup on
run pa8_range_dedup python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition range --dedup on
run mfps python bench.py --steps 20 --warmup 5 --force-ps-path --no-hogwild-probe --exact-steps 0
timeout -k 10 200 python bench/bench_topk.py --steps 10 --warmup 3 > $O/topk.log 2>&1 || { tail -20 $O/topk.log; exit 1; }
echo "topk $(tail -1 $O/topk.log | cut -c1-200)"
timeout -k 10 200 python bench/bench_mf_topk.py --steps 20 --warmup 3 > $O/mftopk.log 2>&1 || { tail -20 $O/mftopk.log; exit 1; }
echo "mftopk $(tail -1 $O/mftopk.log | cut -c1-200)"
timeout -k 10 200 python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash --host-profile $O/pa8_host.txt > $O/pa8_host.log 2>&1 || { tail -20 $O/pa8_host.log; exit 1; }
head -1 $O/pa8_host.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -- python bench.py --steps 20 --warmup 5 --no-hogwild-probe --exact-steps 0 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
echo ALLDONE
