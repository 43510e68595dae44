#!/bin/bash
# conv_glds input-footprint L2 prefetch: bit-identity, then whole-graph A/Bs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split.py -k "l2_prefetch" > gpurun_out/r3_l2pf_test.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv_l2_prefetch --values 0,2 > gpurun_out/r3_ab_l2pf_r18split.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv_l2_prefetch --values 0,1 --dtype fp16 > gpurun_out/r3_ab_l2pf_r18fp16.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv_l2_prefetch --values 0,1 --model resnet50 --batch 1024 --dtype fp16 --iters 10 --rounds 7 > gpurun_out/r3_ab_l2pf_r50fp16.log 2>&1
