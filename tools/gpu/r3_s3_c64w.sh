#!/bin/bash
# layer1 split kernel variants (W32: 2/3, K-split pairs: 4/5): numerics vs fp64, then whole-graph A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split.py -k c64_rows -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_c64w_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_c64_split_variant --values 0,4 > gpurun_out/r3_c64k_ab4.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_c64_split_variant --values 0,5 > gpurun_out/r3_c64k_ab5.log 2>&1
