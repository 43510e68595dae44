#!/bin/bash
# full GPU test suite + bench + kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
stop_if_fatal $? pytest_gpu
tail -3 $OUT/pytest_gpu.log
grep -q "failed\|error" $OUT/pytest_gpu.log && exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1
stop_if_fatal $? bench
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o k -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1
stop_if_fatal $? prof
echo done
