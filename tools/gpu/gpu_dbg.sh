#!/bin/bash
# cluster-consistency diagnosis + stem kernel tests + a short bench + kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 300 python tools/debug_cluster_consistency.py > $OUT/dbg.log 2>&1
stop_if_fatal $? dbg
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -k "stem or runner or window" > $OUT/pt_stem.log 2>&1
stop_if_fatal $? pytest_stem
tail -2 $OUT/pt_stem.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1
stop_if_fatal $? bench
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o k -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1
stop_if_fatal $? prof
echo done
