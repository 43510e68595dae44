#!/bin/bash
# split-fp16 fp32 path: per-layer split tile sweep (ResNet18 b400, ResNet50 b1024)
# + rocprof kernel table of the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -u tools/bench_layers_split.py --batch 400 --json $OUT/layers_split_r18.json > $OUT/layers_split_r18.log 2>&1
stop_if_fatal $? layers18
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_split -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-extras > $OUT/prof_split.log 2>&1
stop_if_fatal $? rocprof
timeout -k 10 400 python -u tools/bench_layers_split.py --model resnet50 --batch 256 --json $OUT/layers_split_r50.json > $OUT/layers_split_r50.log 2>&1
stop_if_fatal $? layers50
echo done
