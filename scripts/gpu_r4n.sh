#!/bin/bash
# Round 4: full GPU suite; top-K / MF+top-K after the launch cuts; emulated N = 2/4/8 with rank-symmetric links.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4n
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=600 step tests python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
for st in length coord lc:1.3; do step topk_$st python bench/bench_topk.py --strategy $st; done
step mf_topk python bench/bench_mf_topk.py
step mf_topk2 python bench/bench_mf_topk.py
step mf_topk_unfused python bench/bench_mf_topk.py --unfused
W=2000 T=500 step emu_links50 python -u bench/bench_emulate_world.py --ws 1,2,4,8 --steps 10 --warmup 3 --link-gbps 50
W=2000 T=500 step emu_links25 python -u bench/bench_emulate_world.py --ws 8 --steps 10 --warmup 3 --link-gbps 25
step w2v_ps python bench/bench_w2v.py --mode standard --ps-path
step prof_w2vps rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2vps -- python bench/bench_w2v.py --mode standard --ps-path --steps 5 --warmup 2
W=600 step hog_emu8 python bench/probe_hogwild.py --users 1250000 --items 1000000 --per-user 51.2 --phases 1 --world 8
step prof_mftopk rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py --steps 6 --warmup 2
echo ALLDONE
