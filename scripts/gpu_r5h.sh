#!/bin/bash
# Round 5: exact user rows with contiguous atomics (tests, bench, emulated N = 8); bench.py --gpus 2 rehearsal on one
# GPU (gloo, FPS_SHARE_GPU=1): the --verify check of the rotation on real kernels.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_hogwild_gpu.py -k "user_modes or atomic" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_tensor_engine_gpu.py -k "mf_ps" -x -v --timeout 200 --timeout-method thread > $O/tests_ps.log 2>&1 || { tail -40 $O/tests_ps.log; exit 1; }
grep -E "PASS|FAIL" $O/tests_ps.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --force-ps-path --no-hogwild-probe > $O/ps_fused_$i.log 2>&1 || { tail -20 $O/ps_fused_$i.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --force-ps-path --no-hogwild-probe --no-fuse-local-push > $O/ps_delta_$i.log 2>&1 || { tail -20 $O/ps_delta_$i.log; exit 1; }
  for v in fused delta; do tail -1 $O/ps_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ps", sys.argv[1], round(d["ms_per_step"],3), "%.4e" % d["value"])' $v; done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ps_fused -- python bench.py --steps 5 --warmup 2 --force-ps-path --no-hogwild-probe > $O/prof_ps_fused.log 2>&1 || { tail -20 $O/prof_ps_fused.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --user-update atomic > $O/bench_atomic.log 2>&1 || { tail -20 $O/bench_atomic.log; exit 1; }
tail -1 $O/bench_atomic.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["user_update"], round(d["ms_per_step"],3), "%.4e" % d["value"], d["config"]["lost_user_update_fraction"], d["effective_updates_per_s"])'
timeout -k 10 300 python bench/bench_emulate_world.py --ws 8 --steps 6 --warmup 2 --user-update atomic > $O/emu8_atomic.log 2>&1 || { tail -20 $O/emu8_atomic.log; exit 1; }
tail -1 $O/emu8_atomic.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_atomic -- python bench.py --steps 3 --warmup 1 --user-update atomic --no-hogwild-probe > $O/prof_atomic.log 2>&1 || { tail -20 $O/prof_atomic.log; exit 1; }
FPS_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 4194304 --no-hogwild-probe > $O/bench_n2_rehearsal.log 2>&1 || { tail -30 $O/bench_n2_rehearsal.log; exit 1; }
grep '^{' $O/bench_n2_rehearsal.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("n2 rehearsal", d["n_gpus"], d["backend"], "verify_ok", d.get("verify_ok"), d["verify"]["verify_max_abs_err_items"], d["verify"]["devices"])'
FPS_SHARE_GPU=1 FPS_VERIFY_MUTANT=wrong_buffer timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --batch 4194304 --no-hogwild-probe > $O/bench_n2_mutant.log 2>&1; echo "mutant rc=$? (expect nonzero)"; grep -c '^{' $O/bench_n2_mutant.log; grep -o "VERIFY FAILED" $O/bench_n2_mutant.log | head -1
echo R5H_DONE
