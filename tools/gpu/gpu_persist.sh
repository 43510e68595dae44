#!/bin/bash
# persistent conv tiles: correctness + layer sweep + cluster GPU test + bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q -k "persistent or tiles" > $OUT/pt_persist.log 2>&1
stop_if_fatal $? pytest_persist
tail -2 $OUT/pt_persist.log
grep -q " passed" $OUT/pt_persist.log && ! grep -q "failed" $OUT/pt_persist.log || exit 1
timeout -k 10 600 python tools/bench_layers.py --batch 400 --rounds 2 --tiles ${TILES:-auto,27,33,36,34,37,41,42,43,44,45,46,47,48} --json $OUT/sweep_persist.json > $OUT/sweep_persist.log 2>&1
stop_if_fatal $? sweep
timeout -k 10 400 python -m pytest tests/test_cluster_gpu.py -x -q > $OUT/pt_cluster.log 2>&1
stop_if_fatal $? pytest_cluster
tail -2 $OUT/pt_cluster.log
echo done
