#!/bin/bash
# split streaming 1x1 conv: numerics vs fp64, whole-forward A/Bs (ResNet50 b1024 and the ResNet18 headline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split.py -k 1x1_stream -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_c1ss_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_split_mask --values 0,15 --model resnet50 --batch 1024 \
    --dtype fp32 --iters 5 --rounds 5 > gpurun_out/r3_c1ss_ab_r50.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_split_mask --values 0,15 --model resnet18 --batch 400 \
    --dtype fp32 > gpurun_out/r3_c1ss_ab_r18.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_mask --values 0,15 --model resnet18 --batch 400 \
    --dtype fp16 > gpurun_out/r3_c1s_ab_r18_fp16.log 2>&1
