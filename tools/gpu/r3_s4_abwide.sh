#!/bin/bash
# A/B: fp16 128x160 tiles at every M (3x3 sweep: 42 beats 36 by 2-13 % on ResNet50 b1024 layers 2-4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_flag.py set_f16_wide_all --model resnet50 --batch 1024 --dtype fp16 --iters 10 --rounds 7 > gpurun_out/r3_ab_f16_wide_all_r50.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_f16_wide_all --dtype fp16 > gpurun_out/r3_ab_f16_wide_all_r18.log 2>&1
