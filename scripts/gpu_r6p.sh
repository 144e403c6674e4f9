#!/bin/bash
# Round 6 (session 2): SGNS N = 8 (hot-owner emulation) kernel trace + host profile; bf16 scorer instruction mix (PMC).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 200 python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3 > $O/w2v8.log 2>&1 || { tail -20 $O/w2v8.log; exit 1; }
tail -1 $O/w2v8.log | cut -c1-400
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2v8 -- python bench/bench_w2v.py --emulate-world 8 --steps 10 --warmup 3 > $O/prof_w2v8.log 2>&1 || { tail -20 $O/prof_w2v8.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w2v1 -- python bench/bench_w2v.py --ps-path --steps 10 --warmup 3 > $O/prof_w2v1.log 2>&1 || { tail -20 $O/prof_w2v1.log; exit 1; }
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY"
i=0
for c in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_mftopk_$i -- python bench/bench_mf_topk.py --steps 4 --warmup 1 > $O/pmc_mftopk_$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $O/pmc_mftopk_$i.log; exit 1; }
  echo "pmc $i ok"
done
echo ALLDONE
