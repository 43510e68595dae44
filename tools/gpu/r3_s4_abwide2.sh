#!/bin/bash
# A/B: split 128x160 tiles at every M (ResNet50 b1024 split, ResNet18 b400 split)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_flag.py set_split_wide_all --model resnet50 --batch 1024 --iters 5 --rounds 7 > gpurun_out/r3_ab_split_wide_all_r50.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_split_wide_all > gpurun_out/r3_ab_split_wide_all_r18.log 2>&1
