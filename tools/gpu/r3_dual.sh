#!/bin/bash
# Round 3: dual-conv (fused downsample) tests + A/Bs (fuse_down on the split
# headline, batch_parts on ResNet50 fp16), kernel table of the headline forward.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_split.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/r3_split_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_flag.py --attr fuse_down --rounds 7 > $OUT/r3_ab_fuse_down.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py --attr batch_parts --values 1,8 --model resnet50 --batch 1024 \
    --dtype fp16 --rounds 5 --iters 10 > $OUT/r3_ab_r50_parts8.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py --attr batch_parts --values 1,16 --model resnet50 --batch 1024 \
    --dtype fp16 --rounds 5 --iters 10 > $OUT/r3_ab_r50_parts16.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r3a -o run -- \
    python3 tools/fwd_loop.py --iters 25 > $OUT/r3_prof_fwd.log 2>&1
