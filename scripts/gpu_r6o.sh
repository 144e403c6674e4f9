#!/bin/bash
# Round 6 (session 2): PA N = 8 (hot-owner emulation, hash) host profile + kernel trace; MF + top-K baseline + kernel trace.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 200 python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash --host-profile $O/pa8_host.txt > $O/pa8.log 2>&1 || { tail -20 $O/pa8.log; exit 1; }
tail -1 $O/pa8.log | cut -c1-300
head -3 $O/pa8_host.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pa8 -- python bench/bench_pa.py --emulate-world 8 --steps 40 --warmup 5 --partition hash > $O/prof_pa8.log 2>&1 || { tail -20 $O/prof_pa8.log; exit 1; }
timeout -k 10 200 python bench/bench_mf_topk.py --steps 20 > $O/mftopk.log 2>&1 || { tail -20 $O/mftopk.log; exit 1; }
tail -1 $O/mftopk.log | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py --steps 20 > $O/prof_mftopk.log 2>&1 || { tail -20 $O/prof_mftopk.log; exit 1; }
echo ALLDONE
