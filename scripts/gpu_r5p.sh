#!/bin/bash
# Round 5: pipelined loads in dedup / hash-table / top-k merge kernels -- kernel + PS-path GPU tests, PA / capacity
# benches, MF + top-K profile.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 600 python -u -m pytest -m gpu tests/test_kernels_gpu.py tests/test_tensor_engine_gpu.py tests/test_emb_pairs.py tests/test_pa_fast.py tests/test_touch_sentinel.py tests/test_tensor_ps_dist.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench/bench_pa.py > $O/pa.log 2>&1 || { tail -20 $O/pa.log; exit 1; }
tail -1 $O/pa.log | cut -c1-200
timeout -k 10 300 python bench/bench_pa.py --ps-path > $O/pa_ps.log 2>&1 || { tail -20 $O/pa_ps.log; exit 1; }
tail -1 $O/pa_ps.log | cut -c1-200
timeout -k 10 300 python bench/bench_topk.py --steps 30 --warmup 3 > $O/topk.log 2>&1 || { tail -20 $O/topk.log; exit 1; }
tail -1 $O/topk.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py > $O/prof_mftopk.log 2>&1 || { tail -20 $O/prof_mftopk.log; exit 1; }
tail -1 $O/prof_mftopk.log | cut -c1-200
echo ALLDONE
