#!/bin/bash
# Focused GPU session: selected kernel tests (PYK), then a per-layer sweep (TILES, LAYERS), then optionally the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv3x3_patch_gpu.py -x -q --timeout 120 --timeout-method thread -k "${PYK:-conv}" > $OUT/pytest_sel.log 2>&1
rc=$?; stop_if_fatal $rc pytest_sel; tail -3 $OUT/pytest_sel.log; [ $rc -eq 0 ] || exit 1
if [ -n "${LAYERS:-}" ]; then
  timeout -k 10 400 python -u tools/bench_layers.py --batch 400 --no-stem --tiles "${TILES:-auto}" --layers "$LAYERS" > $OUT/layers_sel.log 2>&1
  stop_if_fatal $? layers; cat $OUT/layers_sel.log
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > $OUT/bench_sel.log 2>&1
  stop_if_fatal $? bench; tail -1 $OUT/bench_sel.log
fi
echo done
