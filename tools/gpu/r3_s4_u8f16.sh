#!/bin/bash
# fp16 exact-u8 stem: numerics, whole-graph A/Bs (HipRunner.stem_u8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem or runner" > gpurun_out/r3_u8f16_test.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py --attr stem_u8 --dtype fp16 > gpurun_out/r3_ab_u8f16_r18.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py --attr stem_u8 --model resnet50 --batch 1024 --dtype fp16 --iters 10 --rounds 7 > gpurun_out/r3_ab_u8f16_r50.log 2>&1
