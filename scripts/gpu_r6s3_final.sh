#!/bin/bash
# Round 6 session 3, final pass: GPU suite + smoke, headline x2, top-K / MF + top-K x2, the N = 8 bench path
# rehearsed on one GPU (8 gloo ranks sharing the card, small shapes), timed-loop kernel profile of the headline.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
  tail -1 $O/bench_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"],3), "%.4e" % d["value"], "lost", round(d["config"]["lost_user_update_fraction"],4), "eff %.4e" % d["effective_updates_per_s"], "exact %.4e" % d.get("exact_updates_per_s",0), round(d.get("exact_ms_per_step", 0), 3))'
done
for r in 1 2; do
  timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_$r.log 2>&1 || { tail -20 $O/topk_$r.log; exit 1; }
  echo "topk $r $(tail -1 $O/topk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
  timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_$r.log 2>&1 || { tail -20 $O/mftopk_$r.log; exit 1; }
  echo "mftopk $r $(tail -1 $O/mftopk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
FPS_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 8 --steps 3 --warmup 1 --batch 1048576 --users 2000000 > $O/share8.log 2>&1 || { tail -30 $O/share8.log; exit 1; }
tail -1 $O/share8.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("share8", d["n_gpus"], d["backend"], d["config"]["exchange"], "verify_ok", d.get("verify_ok"), round(d["ms_per_step"],2))'
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -- python bench.py --steps 20 --warmup 5 --no-hogwild-probe --exact-steps 0 > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
echo ALLDONE
