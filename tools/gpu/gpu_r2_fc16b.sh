#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fc16; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "model or linear or split" > $OUT/tests2.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests2.log; exit 1; }
tail -2 $OUT/tests2.log
timeout -k 10 300 python -u bench.py --model alexnet --batch 500 --dtype fp16 --steps 30 --warmup 5 --no-extras > $OUT/alex16.log 2>&1 || { echo "alex failed"; tail -20 $OUT/alex16.log; exit 1; }
grep "^{" $OUT/alex16.log | cut -c1-200
timeout -k 10 300 python -u tools/ab_linear_split.py --variants 1,auto > $OUT/ab.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab.log; exit 1; }
tail -6 $OUT/ab.log
