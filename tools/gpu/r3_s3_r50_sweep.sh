#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_layers.py --model resnet50 --batch 1024 --rounds 2 --no-stem \
  --tiles auto,18,19,26,27,31,34,35,36,38,42,70,71,72,73 > gpurun_out/r3_r50_tile_sweep.log 2>&1 &&
timeout -k 10 300 python -u tools/conv_epi_ablate.py --r50 > gpurun_out/r3_r50_epi_ablate.log 2>&1
