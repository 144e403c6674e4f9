#!/bin/bash
bash scripts/gpu_r5g.sh && bash scripts/gpu_r5e.sh && bash scripts/gpu_r5f.sh
