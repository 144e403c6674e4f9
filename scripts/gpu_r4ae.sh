#!/bin/bash
# Round 4 counters of the kernels added late in the round: MF + top-K learning side (mf_online_*, index refresh,
# one-launch seen merge, round plan), PA with the world-1 push in the kernel (write map), fused SGNS PS path.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc4b
mkdir -p $O
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
  run mftopk $pass python bench/bench_mf_topk.py --steps 4 --warmup 2
  run pa_ps $pass python bench/bench_pa.py --ps-path --steps 4 --warmup 1
  run w2v_ps $pass python bench/bench_w2v.py --ps-path --steps 3 --warmup 1
done
python scripts/pmc_summary.py $O mftopk,pa_ps,w2v_ps 10 > $O/summary.md 2>&1 || { cat $O/summary.md; exit 1; }
cat $O/summary.md
