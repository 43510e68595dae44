#!/bin/bash
# fp16 256x160 16-wave tile (43): numerics, then per-layer times vs 42 on ResNet50 b1024 / ResNet18 b400
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
IDUNNO_TEST_TILE43=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "tile" > gpurun_out/r3_t43_test.log 2>&1 &&
timeout -k 10 400 python -u tools/bench_layers.py --model resnet50 --batch 1024 --rounds 2 --no-stem \
  --layers b4c1,b7c1,b8c1,b13c1,b14c1,b8c0,b14c0,b13ds --tiles auto,42,43 > gpurun_out/r3_t43_r50.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_layers.py --model resnet18 --batch 400 --rounds 2 --no-stem --tiles auto,42,43 > gpurun_out/r3_t43_r18.log 2>&1
