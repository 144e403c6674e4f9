#!/bin/bash
# Round 6 (session 2, late): GPU test suite + smoke, then the final measurements (one box).
bash scripts/gpu_r6_tests.sh || exit 1
bash scripts/gpu_r6_final3.sh
