#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_conv3x3_patch_gpu.py -x -q > $OUT/pt_sweep2.log 2>&1
stop_if_fatal $? pytest
tail -2 $OUT/pt_sweep2.log
grep -q "failed\|error" $OUT/pt_sweep2.log && exit 1
timeout -k 10 600 python tools/bench_layers.py --batch 400 --rounds 2 --tiles ${TILES:-auto,26,27,33,34,36,37,38,10,15,16,24} --json $OUT/sweep2.json > $OUT/sweep2.log 2>&1
stop_if_fatal $? sweep
grep -v amdgpu.ids $OUT/sweep2.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1
stop_if_fatal $? bench
tail -1 $OUT/bench.log
echo done
