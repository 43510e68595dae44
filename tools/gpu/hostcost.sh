#!/bin/bash
# Coordinator host cost per round on the GPU box's CPUs (gloo dry run, no GPU work):
# N=1 and N=8 plain, then N=8 with the coordinator's driver thread under cProfile
# (thread CPU clock) -> gpurun_out/TAG/drv8.prof.   bash tools/gpu/hostcost.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for n in 1 8; do
  timeout -k 10 300 python -u bench.py --dry-run --system --gpus $n --steps 400 --warmup 10 --sdfs-images 0 \
    --two-job-queries 2 > $OUT/hostcost_n$n.log 2>&1 || exit 15
done
IDUNNO_PROFILE_DRIVER=$OUT/drv8 IDUNNO_PROFILE_DRIVER_CPU=1 timeout -k 10 300 python -u bench.py --dry-run \
  --system --gpus 8 --steps 400 --warmup 10 --sdfs-images 0 --two-job-queries 2 > $OUT/hostcost_n8_prof.log 2>&1 || exit 16
