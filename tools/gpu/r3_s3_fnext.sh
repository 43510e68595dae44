#!/bin/bash
# bottleneck tail + next reduce 1x1 fused: numerics, whole-forward A/B, driver-shaped ResNet50 fp16 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "fused_next or dual or fused_downsample or conv1x1" -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r3_fnext_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py --attr fuse_next_1x1 --values 0,1 --model resnet50 --batch 1024 --dtype fp16 \
    --iters 10 --rounds 5 > gpurun_out/r3_fnext_ab.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model resnet50 --batch 1024 --dtype fp16 --steps 10 --warmup 3 --no-system \
    > gpurun_out/r3_bench_r50_fp16b.log 2>&1
