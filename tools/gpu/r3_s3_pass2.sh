#!/bin/bash
# GPU pass: whole GPU suite, ResNet50 b1024 fp16 bench, ResNet18 headline bench (launcher, N=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model resnet50 --batch 1024 --dtype fp16 --steps 10 --warmup 3 --no-system \
    > gpurun_out/r3_bench_r50_fp16.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-system > gpurun_out/r3_bench_r18.log 2>&1
