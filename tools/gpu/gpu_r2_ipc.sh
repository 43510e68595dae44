#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/ipc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ipc_gpu.py > $OUT/tests.log 2>&1
rc=$?; tail -25 $OUT/tests.log; exit $rc
