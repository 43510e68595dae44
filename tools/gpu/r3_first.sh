#!/bin/bash
# Round 3, first GPU pass: smoke (4 distinct classes), the launcher bench at N=1
# (headline + system + two-job + coordinator failover), runtime GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3_bench.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_cluster_gpu.py tests/test_ipc_gpu.py -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/r3_gpu_cluster.log 2>&1
