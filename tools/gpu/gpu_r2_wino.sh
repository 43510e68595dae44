#!/bin/bash
# Winograd fp32 conv: numerics first (abort on any fault), then per-layer timing and the bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py -k "wino or model or runner" > $OUT/f32w_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 $OUT/f32w_tests.log
grep -E "FAILED|Error" $OUT/f32w_tests.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_layers_f32.py --batch 400 --json $OUT/layers_f32w.json > $OUT/layers_f32w.log 2>&1
rc=$?; echo "[layers] rc=$rc"; sed -n '/^| layer/,$p' $OUT/layers_f32w.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-extras > $OUT/bench_f32w.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -1 $OUT/bench_f32w.log
exit $rc
