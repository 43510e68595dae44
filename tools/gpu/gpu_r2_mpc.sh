#!/bin/bash
# Multi-process cluster on one MI355X: 8 node processes (HIP fp32 executor, SDFS
# source), SIGKILLed workers / coordinator, prefetch on/off A/B with traces.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/mpc; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 420 python -u tools/bench_mp_cluster.py --nodes 8 --prefetch 1 \
    --scenarios overlap,worker:1,worker:4,worker:8,coord:1 --json $OUT/run1.json --trace $OUT/trace_prefetch1.json \
    --log-dir $OUT > $OUT/run1.log 2>&1 || { echo "run1 failed"; tail -30 $OUT/run1.log; exit 1; }
tail -1 $OUT/run1.log | cut -c1-600
timeout -k 10 420 python -u tools/bench_mp_cluster.py --nodes 8 --prefetch 0 \
    --scenarios overlap,coord:4 --json $OUT/run2.json --trace $OUT/trace_prefetch0.json \
    > $OUT/run2.log 2>&1 || { echo "run2 failed"; tail -30 $OUT/run2.log; exit 1; }
tail -1 $OUT/run2.log | cut -c1-600
timeout -k 10 420 python -u tools/bench_mp_cluster.py --nodes 8 --prefetch 1 \
    --scenarios overlap,coord:8 --json $OUT/run3.json > $OUT/run3.log 2>&1 || { echo "run3 failed"; tail -30 $OUT/run3.log; exit 1; }
tail -1 $OUT/run3.log | cut -c1-600
