#!/bin/bash
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/gpu_tests.log
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/b_default.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --force-ps-path > gpurun_out/b_pspipe.log 2>&1 || exit 1
timeout -k 10 300 python bench/bench_w2v.py --steps 10 --warmup 2 > gpurun_out/b_w2v.log 2>&1 || exit 1
timeout -k 10 300 python bench/bench_pa.py --steps 10 --warmup 2 > gpurun_out/b_pa.log 2>&1 || exit 1
for f in b_default b_pspipe b_w2v b_pa; do tail -1 gpurun_out/$f.log | cut -c1-220; done
rocprofv3 -L > gpurun_out/prof/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/pa -- python bench/bench_pa.py --steps 5 --warmup 1 > gpurun_out/prof_pa.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/w2v_pmc -- python bench/bench_w2v.py --steps 3 --warmup 1 > gpurun_out/prof_w2v_pmc.log 2>&1
echo "pmc rc=$?"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/mf_fetch -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_mf_fetch.log 2>&1
echo "pmc2 rc=$?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/mf_write -- python bench.py --steps 5 --warmup 1 > gpurun_out/prof_mf_write.log 2>&1
echo "pmc3 rc=$?"
echo ALLDONE
