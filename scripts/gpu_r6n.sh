#!/bin/bash
# Round 6 (session 2): tile-SGD cost per rating vs users per phase (does a phase whose user rows fit the
# 256 MiB Infinity Cache pay?).  Scaled geometries keep 1M items and 16M / 8M / 4M ratings per phase launch pair.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6n
mkdir -p $O
probe() {  # name, args...
  local n=$1; shift
  timeout -k 10 180 python bench/probe_partition.py --steps 10 "$@" > $O/probe_$n.json 2> $O/probe_$n.err || { tail -20 $O/probe_$n.err; exit 1; }
  echo "$n $(cat $O/probe_$n.json)"
}
probe P4 --user-phases 4
probe P8 --user-phases 8
probe P2 --user-phases 2
probe u5M_P4 --users 5000000 --batch 33554432 --user-phases 4
probe u2.5M_P4 --users 2500000 --batch 16777216 --user-phases 4
probe u1.25M_P4 --users 1250000 --batch 8388608 --user-phases 4
probe u2.5M_P1 --users 2500000 --batch 16777216 --user-phases 1
echo ALLDONE
