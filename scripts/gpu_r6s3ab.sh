#!/bin/bash
# Round 6 session 3: sanity (GPU suite, smoke, headline) then the scorer prefetch-distance A/B.
bash scripts/gpu_r6s3a.sh && bash scripts/gpu_r6s3b.sh
