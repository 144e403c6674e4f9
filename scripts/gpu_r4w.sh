#!/bin/bash
# Round 4: fixed-shape plans -- padding-slot gathers, captured RCCL collectives (one-rank loopback group),
# fixed plans in the virtual world, engine plumbing with / without captured collectives.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4w
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=200 step kern python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "padding or v4"
T=200 step graph python -u -m pytest tests/test_step_graph_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread
T=400 step vw python -u -m pytest tests/test_vworld_gpu.py tests/test_tensor_engine_gpu.py tests/test_tensor_contract_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread
W=3000 step eng_static python -u bench/bench_engine.py --batches 1,64,4096,65536 --seconds 1 --graph
W=3000 step eng_loop_eager python -u bench/bench_engine.py --batches 1,64,4096,65536 --seconds 1 --loopback
W=3000 step eng_loop_graph python -u bench/bench_engine.py --batches 1,64,4096,65536 --seconds 1 --loopback --graph
echo ALLDONE
