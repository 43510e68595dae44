#!/bin/bash
# Round 6: same-process whole-graph A/Bs of HipRunner.route bits (ops.conv2d_split route).
#   bash tools/gpu/r6_route.sh TAG "A,B@BATCH" ...   e.g. "8,0@50" "0,16@50" "8,0@400"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for spec in "$@"; do
  vals=${spec%@*}; b=${spec#*@}
  timeout -k 10 240 python -u tools/ab_flag.py --attr route --values $vals --batch $b \
    > $OUT/ab_route_${vals/,/_}_b$b.log 2>&1 || exit 11
done
