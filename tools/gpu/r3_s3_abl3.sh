#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_flag.py set_split_wide_l3 > gpurun_out/r3_ab_wide_l3.log 2>&1
