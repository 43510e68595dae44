#!/bin/bash
# GPU pass after container re-creation: smoke, GPU suite, driver bench (N=1), then the first hardware run of tile 43
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_s7_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_s7_gpu_tests.log 2>&1 &&
timeout -k 10 420 python -u bench.py > gpurun_out/r3_s7_bench.log 2>&1 &&
IDUNNO_TEST_TILE43=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k "tile" > gpurun_out/r3_s7_t43_test.log 2>&1
