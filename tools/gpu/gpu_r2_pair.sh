#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pair; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/wino_pair_ab.py > $OUT/pair.md 2>&1 || { echo "failed"; tail -20 $OUT/pair.md; exit 1; }
grep -v amdgpu $OUT/pair.md
