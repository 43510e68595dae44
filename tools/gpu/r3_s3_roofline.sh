#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/layer_roofline.py --model resnet50 --batch 1024 --dtype fp16 > gpurun_out/r3_r50_roofline.md 2>&1 &&
timeout -k 10 300 python -u tools/layer_roofline.py --model resnet18 --batch 400 --dtype fp32 > gpurun_out/r3_r18_roofline.md 2>&1
