#!/bin/bash
# Round 6 whole-graph A/Bs of HipRunner batch-part switches and the B=50 kernel table.
#   bash tools/gpu/r6_ab.sh TAG [steps...]    steps: front parts b50prof b400prof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; shift
STEPS=${*:-front parts b50prof}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    front) timeout -k 10 300 python -u tools/ab_flag.py --attr split_front --values 1,2 > $OUT/ab_split_front.log 2>&1 || exit 11 ;;
    parts) timeout -k 10 300 python -u tools/ab_flag.py --attr batch_parts --values 1,2 > $OUT/ab_batch_parts.log 2>&1 || exit 12 ;;
    b50prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/b50prof -o run -- \
               python -u tools/fwd_loop.py --model resnet18 --batch 50 --iters 100 > $OUT/b50prof.log 2>&1 || exit 13 ;;
    b400prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/b400prof -o run -- \
               python -u tools/fwd_loop.py --model resnet18 --batch 400 --iters 30 > $OUT/b400prof.log 2>&1 || exit 14 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
