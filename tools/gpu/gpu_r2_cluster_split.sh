#!/bin/bash
# 2-job cluster (8 in-process nodes, one GPU) with the split-fp16 and the all-f32-MFMA
# fp32 kernels, then the multi-process SIGKILL recovery run.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT/mpc; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
for impl in split f32mfma split; do
  (cd tools && timeout -k 10 300 python -u bench_cluster.py --nodes 8 --images 10000 --fp32-impl $impl \
      --json ../$OUT/cluster_$impl.json > ../$OUT/cluster_$impl.log 2>&1)
  stop_if_fatal $? cluster_$impl
  python3 -c "import json; d=json.load(open('$OUT/cluster_$impl.json')); print('$impl', d['images_per_s'], d['wall_s'], d['query_latency_p50_s'])"
done
timeout -k 10 420 python -u tools/bench_mp_cluster.py --nodes 8 --prefetch 1 \
    --scenarios overlap,worker:1,worker:4,worker:8,coord:1,coord:4 --json $OUT/mpc/run.json \
    --log-dir $OUT/mpc > $OUT/mpc/run.log 2>&1
stop_if_fatal $? mpc
tail -1 $OUT/mpc/run.log | cut -c1-700
echo done
