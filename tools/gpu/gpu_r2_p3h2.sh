#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/p3h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/stem_pack3_f16_sweep.py > $OUT/sweep.log 2>&1 || { echo "failed"; tail -20 $OUT/sweep.log; exit 1; }
grep -v amdgpu $OUT/sweep.log
