#!/bin/bash
# where the split stem's tile time goes (ablation, profiling only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/stem_ablate.py --split > gpurun_out/r3_stem_split_ablate.log 2>&1
