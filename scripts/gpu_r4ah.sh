#!/bin/bash
# Round 4: count kernel counter width A/B (16-bit packed vs 32-bit) on the local headline and the PS path.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4ah
mkdir -p $O
step() { name=$1; shift; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -40 $O/$name.log; exit 1; }; echo "$name: $(grep -v amdgpu.ids $O/$name.log | tail -1 | cut -c1-${W:-200})"; }
for rep in 1 2; do
  step local_auto_$rep python -u bench.py --no-hogwild-probe
  FPS_TP_H16=1 step local_h16_$rep python -u bench.py --no-hogwild-probe
  step ps_auto_$rep python -u bench.py --force-ps-path --no-hogwild-probe
  FPS_TP_H16=0 step ps_h32_$rep python -u bench.py --force-ps-path --no-hogwild-probe
done
FPS_TP_H16=1 step prof_local_h16 rocprofv3 --kernel-trace --stats --output-format csv -d $O/local_h16 -o run -- python -u bench.py --steps 6 --warmup 2 --no-hogwild-probe
echo ALLDONE
