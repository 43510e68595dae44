#!/bin/bash
# full GPU suite + rocprof kernel table of the split fp32 headline
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
stop_if_fatal $? tests
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_split2 -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-extras > $OUT/prof_split2.log 2>&1
stop_if_fatal $? rocprof
echo done
