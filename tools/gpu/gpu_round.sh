#!/bin/bash
# Round check: full GPU test suite, headline bench, kernel profiles of ResNet18 b400 and ResNet50 b1024.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; stop_if_fatal $rc pytest_gpu; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > $OUT/bench.log 2>&1
stop_if_fatal $? bench; tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof18 -o k -- python3 bench.py --steps 20 --warmup 3 > $OUT/prof18.log 2>&1
stop_if_fatal $? prof18
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof50 -o k -- python3 bench.py --model resnet50 --batch 1024 --shard-images 2048 --steps 10 --warmup 3 > $OUT/prof50.log 2>&1
stop_if_fatal $? prof50; tail -1 $OUT/prof50.log
echo done
