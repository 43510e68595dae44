#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_layers_split.py --tiles 26,27,34,36,38,42,15,16,24 > gpurun_out/r3_resweep.log 2>&1
