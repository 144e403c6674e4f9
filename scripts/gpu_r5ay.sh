#!/bin/bash
# Round 5: the online worker consumes the replayed scan results without copies -- tests, rates, launch counts.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5ay
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_static_plan_gpu.py tests/test_topk_bf16_gpu.py tests/test_topk_fast.py tests/test_topk_seen_merge_gpu.py tests/test_topk_tensor_gpu.py tests/test_tensor_engine_gpu.py tests/test_vworld_gpu.py tests/test_multigpu_nccl_gpu.py tests/test_hogwild_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
for r in 1 2 3; do
  timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_$r.log 2>&1 || { tail -20 $O/mftopk_$r.log; exit 1; }
  echo "mftopk $r $(tail -1 $O/mftopk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench/bench_mf_topk.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("kernel launches", sum(int(r["Calls"]) for r in rows), "total ms %.3f" % (sum(float(r["TotalDurationNs"]) for r in rows) / 1e6))
PY
find $O/prof -name "*kernel_trace.csv" -delete
echo ALLDONE
