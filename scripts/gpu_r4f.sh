#!/bin/bash
# Round 4: Hogwild options (store / sc1 / atomic; phases) with per-update loss counts, secondary PS-path benches
# with kernel profiles, top-K strategies, virtual-world N-rank benches (host-timed links), emulated N = 8.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4f
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -20 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-400})"; }
step probe_store python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 4,1
step probe_sc1 python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 4,1 --user-update sc1
step probe_atomic python bench/probe_hogwild.py --users 10000000 --items 1000000 --phases 1 --user-update atomic
W=260 step bench_store python bench.py
W=260 step bench_sc1 python bench.py --user-update sc1
W=260 step bench_p1 python bench.py --user-phases 1
W=260 step bench_p1_sc1 python bench.py --user-phases 1 --user-update sc1
W=260 step bench_atomic python bench.py --user-update atomic --steps 10
W=260 step mf_ps python bench.py --force-ps-path --steps 10
step prof_mfps rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mfps -- python bench.py --force-ps-path --steps 5 --warmup 2
W=260 step w2v_ps python bench/bench_w2v.py --mode standard --ps-path
step prof_w2vps rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2vps -- python bench/bench_w2v.py --mode standard --ps-path --steps 5 --warmup 2
W=260 step w2v_direct python bench/bench_w2v.py --mode standard
W=260 step pa_ps python bench/bench_pa.py --ps-path
step prof_pa rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pa -- python bench/bench_pa.py --ps-path --steps 5 --warmup 1
W=260 step pa_direct python bench/bench_pa.py
for st in length coord lc:1.3; do W=200 step topk_$st python bench/bench_topk.py --strategy $st; done
W=200 step mf_topk python bench/bench_mf_topk.py
for N in 2 4 8; do W=600 T=200 step vworld_n$N python -u bench/bench_vworld.py --world $N --traceback-s 60; done
W=600 T=200 step vworld_n8_d1 python -u bench/bench_vworld.py --world 8 --dilate 1 --traceback-s 60
T=400 step emulate python bench/bench_emulate_world.py --ws 1,8 --steps 10 --warmup 3
echo ALLDONE
