#!/bin/bash
# Round 6 session 3: bf16 scorer with every block's LDS operand reads issued at the start of the stage
# (FPS_SB_CUR2=1; 128 VGPRs, 4 waves / SIMD, 12 B/lane spill) vs the default -- top-K tests under CUR2, same-box A/B;
# then the whole GPU suite + smoke on this build.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3e
mkdir -p $O
FPS_SB_CUR2=1 timeout -k 10 400 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_topk_tensor_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    FPS_SB_CUR2=$v timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk_${v}_$r.log 2>&1 || { tail -20 $O/topk_${v}_$r.log; exit 1; }
    echo "topk cur2=$v $r $(tail -1 $O/topk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"], d["exact_vs_brute_force"])')"
    FPS_SB_CUR2=$v timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_${v}_$r.log 2>&1 || { tail -20 $O/mftopk_${v}_$r.log; exit 1; }
    echo "mftopk cur2=$v $r $(tail -1 $O/mftopk_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
  done
done
# the whole GPU suite and the smoke on this (final) build, default knobs
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { grep -E "FAILED|Error" $O/suite.log | head -20; tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo ALLDONE
