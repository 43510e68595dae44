#!/bin/bash
# Round 3: staggered DMA issue split tiles (46/47/48) and the 3-stage 128x256 ring (49)
# vs the defaults (36/42), per ResNet18 layer at B=400.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_split.py -x -q -k "tiles" --timeout 120 --timeout-method thread \
    > $OUT/r3_stagger_tests.log 2>&1 &&
timeout -k 10 500 python -u tools/bench_layers_split.py --tiles 36,46,42,48,47,49 > $OUT/r3_stagger_layers.log 2>&1
