#!/bin/bash
set -e
mkdir -p gpurun_out/bucket
for b in 65536 262144 1048576; do
  timeout -k 10 300 python bench/bench_mf_topk.py --bucket $b > gpurun_out/bucket/b$b.json
  python -c "import json; d=json.loads(open('gpurun_out/bucket/b$b.json').read().strip().splitlines()[-1]); print($b, d['value'], d['ms_per_step'])"
done
for b in 65536 1048576; do
  timeout -k 10 300 python bench/bench_topk.py --bucket $b > gpurun_out/bucket/t$b.json
  python -c "import json; d=json.loads(open('gpurun_out/bucket/t$b.json').read().strip().splitlines()[-1]); print('topk', $b, d['value'], d['ms_per_step'])"
done
