#!/bin/bash
# Round 4: full GPU validation, headline bench, Hogwild probe at headline density, virtual-world N-rank benches.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4d
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_touch_sentinel.py -m gpu -x -q -k "tile_partition or delta_mode or sentinel or pulled_features" --timeout 150 --timeout-method thread > gpurun_out/r4d/partition_tests.log 2>&1 || { tail -30 gpurun_out/r4d/partition_tests.log; exit 1; }
tail -1 gpurun_out/r4d/partition_tests.log
timeout -k 10 300 python -u -m pytest tests/test_topk_bf16_gpu.py tests/test_sgns_sampling.py -m gpu -x -q -k "coord or steady_state" --timeout 150 --timeout-method thread > gpurun_out/r4d/coord_tests.log 2>&1 || { tail -30 gpurun_out/r4d/coord_tests.log; exit 1; }
tail -1 gpurun_out/r4d/coord_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r4d/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4d/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r4d/bench_n1.log 2>&1 || { tail -20 gpurun_out/r4d/bench_n1.log; exit 1; }
tail -1 gpurun_out/r4d/bench_n1.log | cut -c1-300
timeout -k 10 300 python bench/probe_hogwild.py --phases 1,4 > gpurun_out/r4d/hogwild.log 2>&1 || { tail -20 gpurun_out/r4d/hogwild.log; exit 1; }
cat gpurun_out/r4d/hogwild.log
timeout -k 10 300 python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 4 > gpurun_out/r4d/hogwild_full.log 2>&1 || { tail -20 gpurun_out/r4d/hogwild_full.log; exit 1; }
cat gpurun_out/r4d/hogwild_full.log
for N in 2 4 8; do
  timeout -k 10 300 python bench/bench_vworld.py --world $N > gpurun_out/r4d/vworld_n$N.log 2>&1 || { tail -20 gpurun_out/r4d/vworld_n$N.log; exit 1; }
  tail -1 gpurun_out/r4d/vworld_n$N.log
done
timeout -k 10 300 python bench/bench_vworld.py --world 8 --dilate 1 > gpurun_out/r4d/vworld_n8_d1.log 2>&1 || { tail -20 gpurun_out/r4d/vworld_n8_d1.log; exit 1; }
tail -1 gpurun_out/r4d/vworld_n8_d1.log
timeout -k 10 300 python bench.py --force-ps-path --steps 10 > gpurun_out/r4d/mf_ps.log 2>&1 || { tail -20 gpurun_out/r4d/mf_ps.log; exit 1; }
tail -1 gpurun_out/r4d/mf_ps.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d/prof_mfps -- python bench.py --force-ps-path --steps 5 --warmup 2 > gpurun_out/r4d/prof_mfps.log 2>&1 || { tail -20 gpurun_out/r4d/prof_mfps.log; exit 1; }
timeout -k 10 300 python bench/bench_w2v.py --mode standard --ps-path > gpurun_out/r4d/w2v_ps.log 2>&1 || { tail -20 gpurun_out/r4d/w2v_ps.log; exit 1; }
tail -1 gpurun_out/r4d/w2v_ps.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d/prof_w2vps -- python bench/bench_w2v.py --mode standard --ps-path --steps 5 --warmup 2 > gpurun_out/r4d/prof_w2vps.log 2>&1 || { tail -20 gpurun_out/r4d/prof_w2vps.log; exit 1; }
timeout -k 10 600 python bench/bench_emulate_world.py --ws 1,8 --steps 10 --warmup 3 > gpurun_out/r4d/emulate.log 2>&1 || { tail -20 gpurun_out/r4d/emulate.log; exit 1; }
tail -3 gpurun_out/r4d/emulate.log
for st in length coord lc:1.3; do
  timeout -k 10 300 python bench/bench_topk.py --strategy $st > gpurun_out/r4d/topk_$st.log 2>&1 || { tail -20 gpurun_out/r4d/topk_$st.log; exit 1; }
  echo "topk $st $(tail -1 gpurun_out/r4d/topk_$st.log | cut -c1-150)"
done
timeout -k 10 300 python bench/bench_pa.py --ps-path > gpurun_out/r4d/pa_ps.log 2>&1 || { tail -20 gpurun_out/r4d/pa_ps.log; exit 1; }
tail -1 gpurun_out/r4d/pa_ps.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d/prof_pa -- python bench/bench_pa.py --ps-path --steps 5 --warmup 1 > gpurun_out/r4d/prof_pa.log 2>&1 || { tail -20 gpurun_out/r4d/prof_pa.log; exit 1; }
echo ALLDONE
