#!/bin/bash
# Secondary configs + cluster bench in one GPU call, each step bounded so the
# whole script stays well inside gpurun's 1200 s cap.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 240 python bench.py --model alexnet --batch 500 --steps 30 --warmup 5 > $OUT/bench_alexnet.log 2>&1
stop_if_fatal $? bench_alexnet
tail -1 $OUT/bench_alexnet.log
timeout -k 10 240 python bench.py --model resnet50 --batch 1024 --shard-images 2048 --steps 20 --warmup 3 > $OUT/bench_r50.log 2>&1
stop_if_fatal $? bench_r50
tail -1 $OUT/bench_r50.log
(cd tools && timeout -k 10 400 python bench_cluster.py --nodes 8 --images 10000 --json ../$OUT/cluster.json > ../$OUT/cluster.log 2>&1)
stop_if_fatal $? cluster
tail -3 $OUT/cluster.log
echo done
