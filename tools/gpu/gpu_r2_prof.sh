#!/bin/bash
# fp32 path: per-layer tile sweep + rocprof kernel table of the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 300 python -u tools/bench_layers_f32.py --batch 400 --torch --json $OUT/layers_f32.json > $OUT/layers_f32.log 2>&1
stop_if_fatal $? layers
tail -25 $OUT/layers_f32.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof32 -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-extras > $OUT/prof32.log 2>&1
stop_if_fatal $? rocprof
echo done
