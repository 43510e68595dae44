#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ne 0 ]; then exit "$rc"; fi; }
timeout -k 10 200 python -u -m pytest tests/test_split.py -x -q --timeout 60 --timeout-method thread -k "c64 or model" > $OUT/c64_tests.log 2>&1
stop_if_fatal $? tests
timeout -k 10 300 python -u tools/bench_layers_split.py --batch 50 --tiles 26,27,34,36,50 > $OUT/layers_b50.log 2>&1
stop_if_fatal $? layers50
for impl in split f32mfma split f32mfma; do
  (cd tools && timeout -k 10 300 python -u bench_cluster.py --nodes 8 --images 10000 --fp32-impl $impl \
      --json ../$OUT/cluster_$impl.json > ../$OUT/cluster_$impl.log 2>&1)
  stop_if_fatal $? cluster_$impl
  python3 -c "import json; d=json.load(open('$OUT/cluster_$impl.json')); print('$impl', d['images_per_s'], d['wall_s'], d['query_latency_p50_s'])"
done
echo done
