#!/bin/bash
# resident-weight 64->64 3x3 conv (tile 50): correctness, then layer1 timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -m pytest tests/test_conv3x3_patch_gpu.py -x -q -k resident > $OUT/pt_c64.log 2>&1
stop_if_fatal $? pytest_c64
tail -3 $OUT/pt_c64.log
grep -q "failed\|error" $OUT/pt_c64.log && exit 1
timeout -k 10 300 python tools/bench_layers.py --batch 400 --rounds 3 --no-stem --layers b0c0,b0c1+res --tiles auto,27,37,40,50 > $OUT/sweep_c64.log 2>&1
stop_if_fatal $? sweep
grep -v amdgpu.ids $OUT/sweep_c64.log
echo done
