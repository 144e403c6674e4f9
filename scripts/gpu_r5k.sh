#!/bin/bash
# Round 5: 256-B row updates -- plain RMW vs float atomics (scopes, XCD-owned rows)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5k
FPS_PROBE_ROWS=1 timeout -k 10 300 python -u bench/probe_atomics.py > gpurun_out/r5k/rows.jsonl 2>&1 || { tail -20 gpurun_out/r5k/rows.jsonl; exit 1; }
cat gpurun_out/r5k/rows.jsonl
