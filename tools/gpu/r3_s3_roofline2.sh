#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/layer_roofline.py --model resnet50 --batch 1024 --dtype fp16 > gpurun_out/r3_r50_roofline2.md 2>&1 &&
timeout -k 10 400 python -u bench.py --model resnet50 --batch 1024 --dtype fp32 --steps 10 --warmup 3 --no-system \
    > gpurun_out/r3_bench_r50_fp32.log 2>&1
