#!/bin/bash
# Round-4 multi-rank rehearsal on a one-GPU box (adds fixed-shape plans and the PA PS path at 2 ranks): 2 and 4 ranks share cuda:0 over gloo (host-staged
# transport) and run bench.py end to end (tiled SGD + item-block ring rotation + user
# phases, and the PS exchange), plus the tiled GPU tests.
set -e
mkdir -p gpurun_out/rehearse4
export TMPDIR=/tmp FPS_SHARE_GPU=1
timeout -k 10 300 python -u -m pytest tests/test_mf_tiled_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rehearse4/tiled_tests.log 2>&1 || { tail -30 gpurun_out/rehearse4/tiled_tests.log; exit 1; }
tail -1 gpurun_out/rehearse4/tiled_tests.log
timeout -k 10 300 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 4194304 > gpurun_out/rehearse4/share2.log 2>&1 || { tail -30 gpurun_out/rehearse4/share2.log; exit 1; }
tail -1 gpurun_out/rehearse4/share2.log | cut -c1-400
timeout -k 10 300 python bench.py --gpus 2 --steps 4 --warmup 1 --batch 4194304 --exchange ps > gpurun_out/rehearse4/share2ps.log 2>&1 || { tail -30 gpurun_out/rehearse4/share2ps.log; exit 1; }
tail -1 gpurun_out/rehearse4/share2ps.log | cut -c1-400
timeout -k 10 300 python bench.py --gpus 4 --steps 3 --warmup 1 --batch 2097152 --users 2000000 > gpurun_out/rehearse4/share4.log 2>&1 || { tail -30 gpurun_out/rehearse4/share4.log; exit 1; }
tail -1 gpurun_out/rehearse4/share4.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench/bench_mf_topk.py --users 100000 --items 200000 --batch 1024 --steps 3 --warmup 1 > gpurun_out/rehearse4/mftopk2.log 2>&1 || { tail -30 gpurun_out/rehearse4/mftopk2.log; exit 1; }
tail -1 gpurun_out/rehearse4/mftopk2.log | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench/bench_pa.py --steps 4 --warmup 1 > gpurun_out/rehearse4/pa2.log 2>&1 || { tail -30 gpurun_out/rehearse4/pa2.log; exit 1; }
tail -1 gpurun_out/rehearse4/pa2.log | cut -c1-300

timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29545 bench/bench_engine.py --batches 64,4096 --seconds 0.5 --capacity > gpurun_out/rehearse4/engine2_fixed.log 2>&1 || { tail -30 gpurun_out/rehearse4/engine2_fixed.log; exit 1; }
tail -1 gpurun_out/rehearse4/engine2_fixed.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29547 bench/bench_pa.py --steps 4 --warmup 1 --ps-path > gpurun_out/rehearse4/pa2ps.log 2>&1 || { tail -30 gpurun_out/rehearse4/pa2ps.log; exit 1; }
tail -1 gpurun_out/rehearse4/pa2ps.log | cut -c1-300
echo ALLDONE
