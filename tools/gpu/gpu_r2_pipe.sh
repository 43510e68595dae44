#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pipe; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cluster_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras > $OUT/raw.log 2>&1 || { echo "raw failed"; tail -20 $OUT/raw.log; exit 1; }
tail -1 $OUT/raw.log | cut -c1-200
timeout -k 10 300 python -u bench.py --system --steps 20 --warmup 5 > $OUT/sys.log 2>&1 || { echo "sys failed"; tail -20 $OUT/sys.log; exit 1; }
tail -1 $OUT/sys.log | cut -c1-200
timeout -k 10 300 python -u bench.py --system --dtype fp16 --steps 20 --warmup 5 > $OUT/sys16.log 2>&1 || { echo "sys16 failed"; tail -20 $OUT/sys16.log; exit 1; }
tail -1 $OUT/sys16.log | cut -c1-200
