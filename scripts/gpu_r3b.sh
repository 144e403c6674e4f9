#!/bin/bash
# Round 3: kernel cleanup + bidirectional rotation on the GPU: kernel / tiled / multi-rank tests,
# per-GPU step of the emulated N = 2/4/8 rotation, headline bench, gloo rehearsal at 2/4/8 ranks.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_mf_tiled_gpu.py tests/test_multirank_gpu.py \
  tests/test_topk_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3b/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r3b/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r3b/bench_n1.log 2>&1 || { tail -20 gpurun_out/r3b/bench_n1.log; exit 1; }
tail -1 gpurun_out/r3b/bench_n1.log | cut -c1-200
timeout -k 10 400 python bench/bench_emulate_world.py --ws 1,2,4,8 > gpurun_out/r3b/emulate_bidir.jsonl 2>&1 || { tail -20 gpurun_out/r3b/emulate_bidir.jsonl; exit 1; }
cat gpurun_out/r3b/emulate_bidir.jsonl
timeout -k 10 400 python bench/bench_emulate_world.py --ws 2,4,8 --rotation ring > gpurun_out/r3b/emulate_ring.jsonl 2>&1 || { tail -20 gpurun_out/r3b/emulate_ring.jsonl; exit 1; }
cat gpurun_out/r3b/emulate_ring.jsonl
export FPS_SHARE_GPU=1
timeout -k 10 300 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 4194304 > gpurun_out/r3b/share2.log 2>&1 || { tail -30 gpurun_out/r3b/share2.log; exit 1; }
tail -1 gpurun_out/r3b/share2.log | cut -c1-200
timeout -k 10 400 python bench.py --gpus 8 --steps 3 --warmup 1 --batch 1048576 --users 2000000 > gpurun_out/r3b/share8.log 2>&1 || { tail -30 gpurun_out/r3b/share8.log; exit 1; }
tail -1 gpurun_out/r3b/share8.log | cut -c1-200
echo ALLDONE
