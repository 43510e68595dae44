#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/v5; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py -k "wino" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u tools/wino_variants.py 3 6 > $OUT/var.md 2>&1 || { echo "var failed"; tail -20 $OUT/var.md; exit 1; }
grep -v amdgpu $OUT/var.md
