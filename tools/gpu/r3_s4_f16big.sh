#!/bin/bash
# fp16 3x3 / strided convs at ResNet50 b1024 and ResNet18 b400: big tiles (256x128, 128x256) after the buffer-DMA rewrite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_layers.py --model resnet50 --batch 1024 --rounds 2 --no-stem \
  --layers b3c1,b4c1,b7c1,b8c1,b13c1,b14c1,b3ds,b7ds,b13ds,b8c0,b14c0 \
  --tiles auto,36,42,10,14,17,21,22,25,30,39 > gpurun_out/r3_s4_f16big_r50.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_layers.py --model resnet18 --batch 400 --rounds 2 --no-stem \
  --tiles auto,36,42,14,25,30 > gpurun_out/r3_s4_f16big_r18.log 2>&1
