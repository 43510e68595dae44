#!/bin/bash
# Cluster-level GPU runs: two concurrent jobs on 8 node processes, the same with a
# mid-job coordinator kill, and the worker / coordinator recovery-time sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
(cd tools && timeout -k 10 400 python -u bench_cluster.py --nodes 8 --images 10000 --json ../$OUT/cluster.json > ../$OUT/cluster.log 2>&1)
stop_if_fatal $? cluster; tail -2 $OUT/cluster.log
(cd tools && timeout -k 10 400 python -u bench_cluster.py --nodes 8 --images 10000 --kill-coordinator-at-frac 0.3 --watchdog 150 --json ../$OUT/cluster_failover.json > ../$OUT/cluster_failover.log 2>&1)
stop_if_fatal $? cluster_failover; tail -2 $OUT/cluster_failover.log
if [ "${RECOVERY:-1}" = "1" ]; then
  timeout -k 10 600 python -u tools/bench_recovery.py --executor hip --nodes 8 --tasks 1,2,4,8 --json $OUT/recovery.json > $OUT/recovery.log 2>&1
  stop_if_fatal $? recovery; tail -2 $OUT/recovery.log
fi
echo done
