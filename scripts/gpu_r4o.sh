#!/bin/bash
# Round 4: counters of the bf16 top-K scorer (LENGTH scan, 4096 queries x 1M items): what bounds it at ~19 % MFMA.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_topk4
mkdir -p $O
pass() {  # name counters...
  name=$1; shift
  rm -rf $O/$name
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$name -- python bench/bench_topk.py --strategy length --steps 3 --warmup 1 > $O/$name.log 2>&1 || { echo "FAIL $name"; tail -5 $O/$name.log; exit 1; }
  echo "$name ok"
}
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
pass p3 FETCH_SIZE
pass p4 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TD_BUSY_avr
pass p2 SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD
python - <<'PY' > $O/summary.txt
import csv, glob, collections
for p in ("p1", "p2", "p3", "p4"):
    fs = glob.glob(f"gpurun_out/pmc_topk4/{p}/*/*counter_collection.csv")
    if not fs:
        continue
    f = fs[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:50]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for k in sorted(agg, key=lambda k: -sum(dur[k].values()))[:3]:
        print(p, k, f"t={sum(dur[k].values())*1e3:.3f}ms n={len(dur[k])}", {c: round(v) for c, v in agg[k].items()})
PY
cat $O/summary.txt
echo ALLDONE
