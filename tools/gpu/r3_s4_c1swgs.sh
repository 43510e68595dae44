#!/bin/bash
# streaming 1x1: more resident workgroups per CU (3 / 4) vs two waves per SIMD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_wgs --values 0,4 --model resnet50 --batch 1024 --dtype fp16 --iters 10 --rounds 7 > gpurun_out/r3_ab_c1s_wgs4_fp16.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_wgs --values 0,3 --model resnet50 --batch 1024 --dtype fp16 --iters 10 --rounds 7 > gpurun_out/r3_ab_c1s_wgs3_fp16.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_stream_wgs --values 0,4 --model resnet50 --batch 1024 --iters 5 --rounds 7 > gpurun_out/r3_ab_c1s_wgs4_split.log 2>&1
