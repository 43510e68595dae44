#!/bin/bash
# conv_glds with buffer-resource DMA: tile numerics (fp16 all ids, split), per-layer split table, headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_split.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r3_bufdma_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_layers_split.py --tiles 36,42 > gpurun_out/r3_bufdma_layers.log 2>&1 &&
timeout -k 10 420 python -u bench.py --no-system > gpurun_out/r3_bufdma_bench.log 2>&1
