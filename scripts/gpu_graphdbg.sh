cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dbg
timeout -k 10 300 python -u -m pytest tests/test_step_graph_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dbg/graph.log 2>&1; tail -60 gpurun_out/dbg/graph.log | grep -v "^$" | tail -45
