#!/bin/bash
# Round 4 final validation: full GPU suite, smoke, headline, secondary benches (fused PS paths, top-K).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4ai
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-400})"; }
T=600 step tests python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
W=1500 step bench python bench.py
W=600 step mf_ps python bench.py --force-ps-path --steps 10 --no-hogwild-probe
W=300 step pa_ps python bench/bench_pa.py --ps-path
W=300 step pa_direct python bench/bench_pa.py
W=300 step w2v_direct python bench/bench_w2v.py --mode standard
W=300 step w2v_ps python bench/bench_w2v.py --mode standard --ps-path
W=300 step topk python bench/bench_topk.py --strategy length
W=300 step mftopk python bench/bench_mf_topk.py
echo ALLDONE
