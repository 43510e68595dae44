#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split.py -k "1x1_stream or dual_split" -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r3_sw_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "
import sys; sys.argv=['x']
from idunno import ops; ops.load().set_conv1x1_split_wide(True)
import pytest; sys.exit(pytest.main(['tests/test_split.py','-k','1x1_stream or dual_split','-x','-q','-p','no:cacheprovider']))
" > gpurun_out/r3_sw_tests_wide.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_flag.py set_conv1x1_split_wide --model resnet50 --batch 1024 --dtype fp32 \
    --iters 5 --rounds 5 > gpurun_out/r3_sw_ab.log 2>&1
