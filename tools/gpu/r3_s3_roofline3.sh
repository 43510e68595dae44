#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/layer_roofline.py --model resnet50 --batch 1024 --dtype fp32 > gpurun_out/r3_r50_split_roofline.md 2>&1
