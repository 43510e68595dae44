#!/bin/bash
# fused split AlexNet stem: numerics, AlexNet split E2E, same-process A/B vs the 3-pass stem
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_split.py \
  -m gpu -k "alex" > gpurun_out/astem_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/ab_flag.py --attr fuse_stem --model alexnet --batch 500 \
  > gpurun_out/astem_ab.log 2>&1
