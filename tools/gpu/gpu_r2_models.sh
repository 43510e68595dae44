#!/bin/bash
# fp32 AlexNet b500 / ResNet50 b1024 benches + kernel tables.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/models; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/alex -o run -- \
    python3 bench.py --model alexnet --batch 500 --steps 10 --warmup 3 --no-extras > $OUT/alex.log 2>&1 || { echo "alex failed"; tail -20 $OUT/alex.log; exit 1; }
tail -1 $OUT/alex.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r50 -o run -- \
    python3 bench.py --model resnet50 --batch 1024 --steps 5 --warmup 2 --no-extras > $OUT/r50.log 2>&1 || { echo "r50 failed"; tail -20 $OUT/r50.log; exit 1; }
tail -1 $OUT/r50.log | cut -c1-400
