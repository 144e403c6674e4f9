#!/bin/bash
# End-of-round secondary benches on the final build: LEMP top-K, online MF + top-K, word2vec SGNS.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fin
timeout -k 10 300 python -u bench/bench_topk.py > gpurun_out/fin/topk.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench/bench_mf_topk.py > gpurun_out/fin/mftopk.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench/bench_w2v.py > gpurun_out/fin/w2v.json 2>/dev/null || exit 1
for f in topk mftopk w2v; do echo "$f $(tail -1 gpurun_out/fin/$f.json | cut -c1-200)"; done
