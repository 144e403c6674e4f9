#!/bin/bash
bash scripts/gpu_r5x.sh && bash scripts/gpu_r5y.sh
