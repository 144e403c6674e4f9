#!/bin/bash
# Round 6: partition id guard (kernel tests), tiled MF tests, bench, link-sleep probe under load.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "tile_partition or mf_sgd" --timeout 200 --timeout-method thread > $O/tests_k.log 2>&1 || { tail -40 $O/tests_k.log; exit 1; }
tail -1 $O/tests_k.log
timeout -k 10 600 python -u -m pytest tests/test_mf_tiled_gpu.py tests/test_hogwild_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_mf.log 2>&1 || { tail -40 $O/tests_mf.log; exit 1; }
tail -1 $O/tests_mf.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", round(d["ms_per_step"],3), "%.4e" % d["value"], d["config"]["lost_user_update_fraction"], "exact %.4e" % d.get("exact_updates_per_s",0), d.get("exact_ms_per_step"))'
timeout -k 10 200 python bench/probe_sleep_under_load.py > $O/sleep.log 2>&1 || { tail -20 $O/sleep.log; exit 1; }
tail -1 $O/sleep.log
echo ALLDONE
