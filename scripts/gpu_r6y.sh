#!/bin/bash
# Round 6 (session 2): the emulated links write the receive during the transfer (second stream) instead of after it.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vworld_gpu.py tests/test_emulated_hot_owner.py tests/test_rotation.py tests/test_tensor_engine.py tests/test_kernels_gpu.py::test_segment_fill_lasts_its_link_time tests/test_kernels_gpu.py::test_segment_fill_matches_torch -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench/bench_emulate_world.py --ws 2,4,8 --steps 20 --warmup 5 --link-gbps 50 > $O/emu_links_$r.jsonl 2>$O/emu_links_$r.err || { tail -20 $O/emu_links_$r.err; exit 1; }
  python - $O/emu_links_$r.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print("emu_links", d["emulated_world"], round(d["ms_per_step"], 3), "%.3e" % d["updates_per_s_per_gpu"], round(d["comm_wait_ms_per_step"], 3))
PY
done
run() {  # name, cmd...
  local n=$1; shift
  timeout -k 10 200 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4g" % d.get("per_gpu_rate", d["value"]), "wait", d.get("exposed_wait_ms_per_step"))')"
}
for n in 8; do
  run pa${n}_hash python bench/bench_pa.py --emulate-world $n --steps 40 --warmup 5 --partition hash
  run pa${n}_range python bench/bench_pa.py --emulate-world $n --steps 40 --warmup 5 --partition range
  run w2v$n python bench/bench_w2v.py --emulate-world $n --steps 10 --warmup 3
done
run cap8 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8
run cap8_bf16 python bench/bench_capacity.py --steps 20 --warmup 3 --emulate-world 8 --wire bf16
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof4 -- python bench/bench_emulate_world.py --ws 4 --steps 6 --warmup 3 --link-gbps 50 > $O/prof4.log 2>&1 || { tail -20 $O/prof4.log; exit 1; }
echo ALLDONE
