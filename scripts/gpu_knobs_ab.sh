#!/bin/bash
# Earlier A/B knobs re-run with the final partition defaults (non-temporal scatters, 256k chunks):
# scatter register prefetch (FPS_TP3_PIPE=1), pipelined user-row loads (FPS_MF_PIPE=1), 128-row
# tiles (FPS_TILE_ROWS=128); bench.py alternating on one box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/knobs
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py > gpurun_out/knobs/b_$name.$rep.log 2>&1 || { tail -20 gpurun_out/knobs/b_$name.$rep.log; exit 1; }
  python -c "import json; d = json.loads(open('gpurun_out/knobs/b_$name.$rep.log').read().strip().splitlines()[-1]); print('$name rep$rep', round(d['value'] / 1e9, 3), round(d['ms_per_step'], 3))"
}
for rep in 1 2; do
  run default FPS_NONE=1
  run tp3pipe FPS_TP3_PIPE=1
  run mfpipe FPS_MF_PIPE=1
  run rows128 FPS_TILE_ROWS=128
done
