#!/bin/bash
# Round-2 fp32 path: kernel numerics, then a short headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py \
  > gpurun_out/f32_tests.log 2>&1
rc=$?
tail -5 gpurun_out/f32_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_f32.log 2>&1
rc2=$?
tail -3 gpurun_out/bench_f32.log
exit $rc2
