#!/bin/bash
# fused-next 1x1 with LDS-staged residual / y / z: numerics, then whole-graph A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fused_next or conv1x1" > gpurun_out/r3_lion2_test.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_lio_n2 --model resnet50 --batch 1024 --dtype fp16 --iters 10 --rounds 7 > gpurun_out/r3_ab_lion2_fp16.log 2>&1
