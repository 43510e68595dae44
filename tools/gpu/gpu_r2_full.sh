#!/bin/bash
# Full GPU test suite + smoke + headline bench (round-end rehearsal).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $OUT/gpu_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -5 $OUT/gpu_tests.log; grep -E "^FAILED|^ERROR" $OUT/gpu_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "[smoke] rc=$rc"; tail -3 $OUT/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_full.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -1 $OUT/bench_full.log
exit $rc
