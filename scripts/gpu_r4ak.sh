#!/bin/bash
# Round 4 end state: full GPU suite + smoke + headline on the committed tree.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4ak
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -30 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-300})"; }
T=600 step tests python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step smoke python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
W=400 step bench python bench.py
echo ALLDONE
