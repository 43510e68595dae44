#!/bin/bash
# streaming 1x1 conv (tile 80): numerics, ResNet50 per-layer times, whole-forward A/Bs of the shape mask
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k conv1x1_stream -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_c1s_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_layers.py --model resnet50 --batch 1024 --rounds 2 --no-stem --tiles auto,36,42,80 \
    --layers b3ds,b7ds,b13ds,b4c0,b7c0,b13c2+res > gpurun_out/r3_c1s_layers2.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_mask --values 3,7 --model resnet50 --batch 1024 --dtype fp16 \
    --iters 10 --rounds 5 > gpurun_out/r3_c1s_ab_mask7.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_mask --values 3,11 --model resnet50 --batch 1024 --dtype fp16 \
    --iters 10 --rounds 5 > gpurun_out/r3_c1s_ab_mask11.log 2>&1
