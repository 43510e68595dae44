#!/bin/bash
# Round 3: dual conv (long tiles first) microbench + A/Bs: fuse_down, layer1 ring depth 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 250 python -u tools/dual_ab.py > $OUT/r3_dual_ab2.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_flag.py --attr fuse_down --rounds 7 > $OUT/r3_ab_fuse_down2.log 2>&1 &&
timeout -k 10 200 python -u tools/ab_flag.py set_split_c64_depth --values 3,4 --rounds 7 > $OUT/r3_ab_c64_depth.log 2>&1
