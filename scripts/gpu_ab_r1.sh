#!/bin/bash
# Same-box A/B of the headline: round-1 final tree (_ab_r1, a git worktree of 0e1bffa with its
# own kernel build) vs the current tree, alternating, bench.py defaults.
set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
  (cd _ab_r1 && timeout -k 10 300 python bench.py > ../gpurun_out/ab/r1_$rep.json 2>/dev/null)
  python -c "import json; d=json.loads(open('gpurun_out/ab/r1_$rep.json').read().strip().splitlines()[-1]); print('r1', d['value'], d['ms_per_step'])"
  timeout -k 10 300 python bench.py > gpurun_out/ab/r2_$rep.json 2>/dev/null
  python -c "import json; d=json.loads(open('gpurun_out/ab/r2_$rep.json').read().strip().splitlines()[-1]); print('r2', d['value'], d['ms_per_step'])"
done
