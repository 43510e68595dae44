#!/bin/bash
# streaming 1x1 with residual / output through per-wave LDS tiles: numerics, then whole-graph A/Bs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_split.py -k "conv1x1_stream or conv1x1_dual or split_1x1_stream" > gpurun_out/r3_lio_test.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_lio --model resnet50 --batch 1024 --dtype fp16 --iters 10 --rounds 7 > gpurun_out/r3_ab_lio_fp16.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_lio --model resnet50 --batch 1024 --iters 5 --rounds 7 > gpurun_out/r3_ab_lio_split.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_lio > gpurun_out/r3_ab_lio_r18.log 2>&1
