#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fc16; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "linear or split" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/fc_f16_sweep.py > $OUT/fc16.md 2>&1 || { echo "sweep failed"; tail -20 $OUT/fc16.md; exit 1; }
grep -v amdgpu $OUT/fc16.md
