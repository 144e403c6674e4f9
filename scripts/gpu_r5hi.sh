#!/bin/bash
# r5h (exact user rows, fused MF PS push, N = 2 rehearsal), r5i (deferred top-K results), r5j (count-kernel A/B)
bash scripts/gpu_r5h.sh && bash scripts/gpu_r5i.sh && bash scripts/gpu_r5j.sh
