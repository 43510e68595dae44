#!/bin/bash
# split stem, two conv rows per pass: numerics, ablation, whole-graph A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split.py -k stem_split_fused > gpurun_out/r3_rp2_test.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_stem_split_rp2 > gpurun_out/r3_ab_stem_rp2.log 2>&1
