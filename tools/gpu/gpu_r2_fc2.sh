#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fc2; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py -k "linear or model or runner" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-250
timeout -k 10 300 python -u bench.py --model alexnet --batch 500 --steps 20 --warmup 5 --no-extras > $OUT/alex.log 2>&1 || { echo "alex failed"; tail -20 $OUT/alex.log; exit 1; }
tail -1 $OUT/alex.log | cut -c1-250
timeout -k 10 300 python -u bench.py --model resnet50 --batch 1024 --steps 5 --warmup 2 --no-extras > $OUT/r50.log 2>&1 || { echo "r50 failed"; tail -20 $OUT/r50.log; exit 1; }
tail -1 $OUT/r50.log | cut -c1-250
