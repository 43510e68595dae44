#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py -k "wino or model or runner" > $OUT/f32w_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -2 $OUT/f32w_tests.log; grep -E "^FAILED" $OUT/f32w_tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/wino_ablate.py > $OUT/wino_ablate.log 2>&1
rc=$?; echo "[ablate] rc=$rc"; grep "^|" $OUT/wino_ablate.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-extras > $OUT/bench_f32w.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -1 $OUT/bench_f32w.log | cut -c1-300
exit $rc
