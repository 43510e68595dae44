#!/bin/bash
# split bottleneck tail as one GEMM: numerics vs fp64, whole-forward A/B (ResNet50 b1024 fp32 split)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split.py -k "dual_split or split_fused_downsample" -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r3_dual1s_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py --attr fuse_down_1x1 --values 0,1 --model resnet50 --batch 1024 --dtype fp32 \
    --iters 5 --rounds 5 > gpurun_out/r3_dual1s_ab.log 2>&1
