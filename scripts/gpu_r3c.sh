#!/bin/bash
# Round 3 pass: kernel / tiled / multi-rank / SGNS / offline-PA / contract tests, headline bench,
# emulated N-GPU rotation steps, SGNS bench in both modes, gloo rehearsal at 2 and 8 ranks.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py tests/test_multirank_gpu.py \
  tests/test_topk_bf16_gpu.py tests/test_sgns_sampling.py tests/test_pa_offline_tensor_gpu.py \
  tests/test_tensor_contract_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3c/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3c/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r3c/bench_n1.log 2>&1 || { tail -20 gpurun_out/r3c/bench_n1.log; exit 1; }
tail -1 gpurun_out/r3c/bench_n1.log | cut -c1-200
timeout -k 10 400 python bench/bench_emulate_world.py --ws 1,2,4,8 > gpurun_out/r3c/emulate_bidir.jsonl 2>&1 || { tail -20 gpurun_out/r3c/emulate_bidir.jsonl; exit 1; }
cat gpurun_out/r3c/emulate_bidir.jsonl
timeout -k 10 400 python bench/bench_emulate_world.py --ws 2,4,8 --rotation ring > gpurun_out/r3c/emulate_ring.jsonl 2>&1 || { tail -20 gpurun_out/r3c/emulate_ring.jsonl; exit 1; }
cat gpurun_out/r3c/emulate_ring.jsonl
timeout -k 10 300 python bench/bench_w2v.py --mode standard > gpurun_out/r3c/w2v_standard.log 2>&1 || { tail -20 gpurun_out/r3c/w2v_standard.log; exit 1; }
tail -1 gpurun_out/r3c/w2v_standard.log | cut -c1-300
timeout -k 10 300 python bench/bench_w2v.py --mode shared > gpurun_out/r3c/w2v_shared.log 2>&1 || { tail -20 gpurun_out/r3c/w2v_shared.log; exit 1; }
tail -1 gpurun_out/r3c/w2v_shared.log | cut -c1-300
export FPS_SHARE_GPU=1
timeout -k 10 300 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 4194304 > gpurun_out/r3c/share2.log 2>&1 || { tail -30 gpurun_out/r3c/share2.log; exit 1; }
tail -1 gpurun_out/r3c/share2.log | cut -c1-200
timeout -k 10 400 python bench.py --gpus 8 --steps 3 --warmup 1 --batch 1048576 --users 2000000 > gpurun_out/r3c/share8.log 2>&1 || { tail -30 gpurun_out/r3c/share8.log; exit 1; }
tail -1 gpurun_out/r3c/share8.log | cut -c1-200
echo ALLDONE
