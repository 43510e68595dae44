#!/bin/bash
# rocprof kernel table of the fp32 headline forward (current code).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof32b -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-extras > $OUT/prof32b.log 2>&1
rc=$?; echo "[rocprof] rc=$rc"; tail -1 $OUT/prof32b.log
exit $rc
