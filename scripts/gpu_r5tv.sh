#!/bin/bash
bash scripts/gpu_r5t.sh && bash scripts/gpu_validate.sh
