#!/bin/bash
# GPU session focused on kernel performance: numerics, per-layer sweep, vendor baseline, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() {
  local rc=$1
  echo "[$2] rc=$rc"
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then echo "fatal in $2"; exit "$rc"; fi
}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
stop_if_fatal $? pytest_gpu
tail -3 $OUT/pytest_gpu.log
timeout -k 10 400 python tools/bench_layers.py --batch 400 --json $OUT/layers_r18.json > $OUT/layers_r18.log 2>&1
stop_if_fatal $? layers
timeout -k 10 300 python tools/bench_torch_baseline.py --model resnet18 --batch 400 > $OUT/torch_baseline.log 2>&1
stop_if_fatal $? torch_baseline
tail -1 $OUT/torch_baseline.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1
stop_if_fatal $? bench
tail -1 $OUT/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
      python3 bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1
  stop_if_fatal $? rocprof
fi
echo done
