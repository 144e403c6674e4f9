#!/bin/bash
# Round 4: 16-byte gather / apply kernels (SGNS / MF / PA PS paths), geometric top-K segments past the bucket,
# full GPU suite first.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4j
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-400})"; }
T=600 step tests python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
W=300 step w2v_ps python bench/bench_w2v.py --mode standard --ps-path
W=300 step mf_ps python bench.py --force-ps-path --steps 10 --no-hogwild-probe
W=300 step pa_ps python bench/bench_pa.py --ps-path
W=500 step mf_topk python bench/bench_mf_topk.py
W=500 step mf_topk_seed1k python bench/bench_mf_topk.py --seed-items 1024
W=500 step mf_topk_seg64k python bench/bench_mf_topk.py --max-segment 65536
for st in length coord lc:1.3; do W=300 step topk_$st python bench/bench_topk.py --strategy $st; done
step prof_w2vps rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2vps -- python bench/bench_w2v.py --mode standard --ps-path --steps 5 --warmup 2
step prof_mftopk rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mftopk -- python bench/bench_mf_topk.py --steps 6 --warmup 2
echo ALLDONE
