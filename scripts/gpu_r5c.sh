#!/bin/bash
# Round 5: headline after the partition-scan fix (x2) + kernel stats; config #5 on today's TensorPS (25e9 params /
# GPU, Adagrad, staleness 2) + kernel stats; PMC of the local headline with and without the side-stream partition.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-hogwild-probe > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c1-260
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -- python bench.py --steps 5 --warmup 1 --no-hogwild-probe > $O/prof_bench.log 2>&1 || { tail -20 $O/prof_bench.log; exit 1; }
echo "prof ok"
timeout -k 10 600 python -u bench/bench_capacity.py --params-per-gpu 25e9 --staleness 2 --optimizer adagrad > $O/capacity.log 2>&1 || { tail -20 $O/capacity.log; exit 1; }
tail -1 $O/capacity.log | cut -c1-600
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_capacity -- python bench/bench_capacity.py --params-per-gpu 25e9 --staleness 2 --optimizer adagrad --steps 6 --warmup 2 > $O/prof_capacity.log 2>&1 || { tail -20 $O/prof_capacity.log; exit 1; }
echo "prof capacity ok"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
run() {  # name pass cmd...
  name=$1; pass=$2; shift 2
  eval ctr=\$P$pass
  rm -rf $O/${name}_$pass
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/${name}_$pass -- "$@" > $O/${name}_$pass.log 2>&1 || { echo "FAIL $name $pass"; tail -5 $O/${name}_$pass.log; exit 1; }
  echo "$name $pass ok"
}
for pass in 1 2 3; do
  run mf $pass python bench.py --steps 3 --warmup 1 --no-hogwild-probe
  run mfnp $pass python bench.py --steps 3 --warmup 1 --no-hogwild-probe --no-prefetch
done
python scripts/pmc_summary.py $O mf,mfnp 6 > $O/summary.md 2>&1 || { cat $O/summary.md; exit 1; }
cat $O/summary.md
echo ALLDONE
