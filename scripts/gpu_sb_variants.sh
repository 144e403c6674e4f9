#!/bin/bash
# A/B of the bf16 filter kernel shapes (FPS_SB_VARIANT; default = 4 query blocks + mask epilogue): 32-query blocks per wave
# (1 / 2 / 4) and the bit-mask candidate epilogue; numerics of each, then both top-K benches.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sbv
for v in qb2 qb1 qb4 mask; do
  FPS_SB_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_topk_bf16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sbv/tests_$v.log 2>&1 || { tail -30 gpurun_out/sbv/tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/sbv/tests_$v.log)"
done
for rep in 1 2; do
  for v in default qb2 qb1 qb4 mask; do
    FPS_SB_VARIANT=$v timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/sbv/topk_$v.$rep.json 2>/dev/null || exit 1
    FPS_SB_VARIANT=$v timeout -k 10 300 python -u bench/bench_mf_topk.py > gpurun_out/sbv/mftopk_$v.$rep.json 2>/dev/null || exit 1
    python - $v $rep <<'PY'
import json, sys
v, rep = sys.argv[1], sys.argv[2]
a = json.load(open(f"gpurun_out/sbv/topk_{v}.{rep}.json"))
b = json.load(open(f"gpurun_out/sbv/mftopk_{v}.{rep}.json"))
print(f"{v:8s} rep{rep} topk {a['value']:.3e}  mftopk {b['value']:.3e}")
PY
  done
done
