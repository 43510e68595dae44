#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/side; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py -k "side_stream" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/ab_flag.py --attr side_down --dtype fp32 > $OUT/ab_fp32.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_fp32.log; exit 1; }
cat $OUT/ab_fp32.log | grep -v amdgpu
timeout -k 10 300 python -u tools/ab_flag.py --attr side_down --dtype fp16 > $OUT/ab_fp16.log 2>&1 || { echo "ab16 failed"; tail -20 $OUT/ab_fp16.log; exit 1; }
cat $OUT/ab_fp16.log | grep -v amdgpu
