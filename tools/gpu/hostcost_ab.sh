#!/bin/bash
# Same-box A/B of the coordinator host cost (gloo dry run, N=8, system phase only):
# the current tree vs a git worktree (default ab/r5end), alternating, 2 runs each.
#   bash tools/gpu/hostcost_ab.sh TAG [worktree]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; WT=${2:-ab/r5end}
OUT=$PWD/gpurun_out/$TAG; mkdir -p $OUT
ROOT=$PWD
for i in 1 2; do
  for arm in new old; do
    d=$ROOT; [ $arm = old ] && d=$ROOT/$WT
    (cd $d && timeout -k 10 300 python -u bench.py --dry-run --system --gpus 8 --steps 400 --warmup 10 \
      --sdfs-images 0 --two-job-queries 2 > $OUT/hc8_${arm}_$i.log 2>&1) || exit 15
  done
done
