#!/bin/bash
# Round 6 session 3: one-launch round plan (LDS bitonic sort + run scans) -- top-K / seen-merge tests, then the
# online MF + top-K bench x3 and its kernel profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s3d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_topk_seen_merge_gpu.py tests/test_topk_tensor_gpu.py tests/test_topk_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  timeout -k 10 300 python bench/bench_mf_topk.py > $O/mftopk_$r.log 2>&1 || { tail -20 $O/mftopk_$r.log; exit 1; }
  echo "mftopk $r $(tail -1 $O/mftopk_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "%.4e" % d["value"])')"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py --steps 20 --warmup 3 > $O/prof_mftopk.log 2>&1 || { tail -20 $O/prof_mftopk.log; exit 1; }
echo ALLDONE
