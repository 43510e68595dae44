#!/bin/bash
# ResNet50 fp16 / split forward with K=512 streaming 1x1 kernels back on the register path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_split.py -k "conv1x1_stream or split_1x1_stream" > gpurun_out/r3_k512_test.log 2>&1 &&
timeout -k 10 200 python -u tools/fwd_loop.py --model resnet50 --batch 1024 --dtype fp16 --iters 20 > gpurun_out/r3_k512_fwd.log 2>&1 &&
timeout -k 10 200 python -u tools/fwd_loop.py --model resnet50 --batch 1024 --dtype fp32 --iters 10 >> gpurun_out/r3_k512_fwd.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_k512_prof -o run -- \
    python3 tools/fwd_loop.py --model resnet50 --batch 1024 --dtype fp16 --iters 10 > gpurun_out/r3_k512_prof.log 2>&1
