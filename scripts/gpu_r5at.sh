#!/bin/bash
# Round 5 end: full GPU validation, then LEMP / MF + top-K end-to-end rates on the final build.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_validate.sh || exit 1
O=gpurun_out/r5at
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_$r.log 2>&1 || { tail -20 $O/topk_$r.log; exit 1; }
  echo "topk $r $(tail -1 $O/topk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_$r.log 2>&1 || { tail -20 $O/mftopk_$r.log; exit 1; }
  echo "mftopk $r $(tail -1 $O/mftopk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], "%.3e" % d["learning_updates_per_s"])')"
done
echo R5AT_DONE
