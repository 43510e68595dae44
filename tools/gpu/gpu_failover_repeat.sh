#!/bin/bash
# Mid-job coordinator failover (8 nodes on one GPU, two concurrent jobs), repeated
# to catch races, then the plain two-job run and the recovery-time sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for i in ${RUNS:-1 2 3}; do
  (cd tools && timeout -k 10 200 python -u bench_cluster.py --nodes 8 --images 10000 --kill-coordinator-at-frac 0.3 \
      --watchdog 120 --json ../$OUT/cf$i.json > ../$OUT/cf$i.log 2>&1)
  rc=$?; echo "failover $i rc=$rc"; [ $rc -ge 124 ] && exit $rc
done
RECOVERY=${RECOVERY:-0} bash tools/gpu_cluster.sh
