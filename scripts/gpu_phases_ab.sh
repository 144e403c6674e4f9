#!/bin/bash
# User phases P = 4 (auto) vs 5 / 6 / 8 on the headline (needs > 16k partition buckets), alternating, same box.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/phases
for rep in 1 2; do
  for P in 4 6 8 5; do
    timeout -k 10 300 python bench.py --user-phases $P > gpurun_out/phases/p${P}_r$rep.log 2>&1 || { tail -20 gpurun_out/phases/p${P}_r$rep.log; exit 1; }
    echo "P=$P rep=$rep $(tail -1 gpurun_out/phases/p${P}_r$rep.log | cut -c1-160)"
  done
done
echo ALLDONE
