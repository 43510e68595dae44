#!/bin/bash
# conv_big (v3 loop) session: its numerics first, then the per-layer sweep vs the v2 tiles, then the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_big_tiles" > $OUT/pytest_big.log 2>&1
stop_if_fatal $? pytest_big
tail -3 $OUT/pytest_big.log
grep -q " passed" $OUT/pytest_big.log && ! grep -q "failed" $OUT/pytest_big.log || { echo "numerics failed"; exit 1; }
timeout -k 10 400 python -u tools/bench_layers.py --batch 400 --no-stem --tiles "${TILES:-auto,36,34,27,60,61,62,63,65,66,67}" \
   --layers "${LAYERS:-b2c0,b2c1+res,b3c0,b4c0,b4c1+res,b5c0,b6c0,b6c1+res,b7c0}" --json $OUT/layers_big.json > $OUT/layers_big.log 2>&1
stop_if_fatal $? layers
cat $OUT/layers_big.log
echo done
