#!/bin/bash
# register-pooled split stem: numerics, ablation, whole-graph A/Bs (3 and 4 workgroups per CU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split.py -k stem_split_fused > gpurun_out/r3_reg_test.log 2>&1 &&
timeout -k 10 200 python -u tools/stem_ablate.py --split --reg 3 > gpurun_out/r3_stem_reg_ablate.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_stem_split_reg --values 0,3 > gpurun_out/r3_ab_stem_reg3.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_stem_split_reg --values 0,4 > gpurun_out/r3_ab_stem_reg4.log 2>&1
