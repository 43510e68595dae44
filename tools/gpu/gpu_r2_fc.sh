#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/fc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/fc_f32_sweep.py > $OUT/fc.md 2>&1 || { echo "failed"; tail -20 $OUT/fc.md; exit 1; }
grep -v amdgpu $OUT/fc.md
