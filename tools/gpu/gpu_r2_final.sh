#!/bin/bash
# round-2 split-path measurements: headline bench with extras, other models, system mode
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_full.log 2>&1
stop_if_fatal $? bench
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --model alexnet --batch 500 > $OUT/bench_alexnet.log 2>&1
stop_if_fatal $? alexnet
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-extras --model resnet50 --batch 1024 > $OUT/bench_r50.log 2>&1
stop_if_fatal $? r50
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --system > $OUT/bench_system.log 2>&1
stop_if_fatal $? system
echo done
