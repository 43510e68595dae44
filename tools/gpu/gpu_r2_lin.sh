#!/bin/bash
# Winograd LIN blocking: tests, same-box A/B, bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py -k "wino" > $OUT/lin_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/lin_tests.log; exit 1; }
tail -2 $OUT/lin_tests.log
timeout -k 10 200 python -u tools/wino_lin.py > $OUT/wino_lin.md 2>&1 || { echo "ab failed"; tail -20 $OUT/wino_lin.md; exit 1; }
cat $OUT/wino_lin.md
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_lin.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_lin.log; exit 1; }
tail -1 $OUT/bench_lin.log | cut -c1-300
