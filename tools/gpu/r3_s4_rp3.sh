#!/bin/bash
# split stem, three conv rows per pass vs two: numerics and whole-graph A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split.py -k stem_split_fused > gpurun_out/r3_rp3_test.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_stem_split_rp2 --values 2,3 > gpurun_out/r3_ab_stem_rp3.log 2>&1
