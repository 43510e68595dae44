#!/bin/bash
# Round 3 (session 3) GPU pass: smoke, launcher bench at N=1, library ceilings
# for the split conv layers, then the whole GPU test suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 &&
timeout -k 10 420 python -u bench.py > gpurun_out/r3_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/gemm_ceiling.py > gpurun_out/r3_gemm_ceiling.md 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_gpu_tests.log 2>&1
