#!/bin/bash
# Full GPU validation: all GPU tests, headline bench, other configs, cluster + recovery benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 900 python -m pytest tests -m gpu -q > $OUT/pytest_gpu.log 2>&1
stop_if_fatal $? pytest_gpu
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench.log 2>&1
stop_if_fatal $? bench
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --model alexnet --batch 500 --steps 30 --warmup 5 > $OUT/bench_alexnet.log 2>&1
stop_if_fatal $? bench_alexnet
tail -1 $OUT/bench_alexnet.log
timeout -k 10 300 python bench.py --model resnet50 --batch 1024 --shard-images 2048 --steps 20 --warmup 3 > $OUT/bench_r50.log 2>&1
stop_if_fatal $? bench_r50
tail -1 $OUT/bench_r50.log
if [ "${CLUSTER:-1}" = "1" ]; then
  (cd tools && timeout -k 10 600 python bench_cluster.py --nodes 8 --images 10000 --json ../$OUT/cluster.json > ../$OUT/cluster.log 2>&1)
  stop_if_fatal $? cluster
  (cd tools && timeout -k 10 600 python bench_cluster.py --nodes 8 --images 10000 --kill-coordinator-after 0.5 --json ../$OUT/cluster_failover.json > ../$OUT/cluster_failover.log 2>&1)
  stop_if_fatal $? cluster_failover
  timeout -k 10 900 python tools/bench_recovery.py --executor hip --nodes 8 --tasks 1,2,4,8 --json $OUT/recovery.json > $OUT/recovery.log 2>&1
  stop_if_fatal $? recovery
fi
echo done
