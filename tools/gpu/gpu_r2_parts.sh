#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/parts; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py -k "stem_parts or pack3_window" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in 1,2 1,4 1,8; do
timeout -k 10 300 python -u tools/ab_flag.py --attr stem_parts --values $v --dtype fp32 > $OUT/ab_$v.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_$v.log; exit 1; }
grep -v amdgpu $OUT/ab_$v.log
done
