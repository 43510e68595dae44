#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/p3h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pack3_f16_gpu.py tests/test_kernels_f32_gpu.py -k "pack3 or model" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --model alexnet --batch 500 --dtype fp16 --steps 20 --warmup 5 --no-extras > $OUT/alex16.log 2>&1 || { echo "alex failed"; tail -20 $OUT/alex16.log; exit 1; }
grep "^{" $OUT/alex16.log | cut -c1-250
