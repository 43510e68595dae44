#!/bin/bash
# SDFS shard peer copies (HBM -> HBM over IPC): tests + cold-job A/B on 8 node processes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/peer; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cluster_gpu.py tests/test_ipc_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for pc in 1 0; do
timeout -k 10 300 python -u tools/bench_mp_cluster.py --nodes 8 --prefetch 1 --peer-copy $pc --scenarios overlap \
    --json $OUT/peer$pc.json --trace $OUT/trace_peer$pc.json > $OUT/peer$pc.log 2>&1 || { echo "run $pc failed"; tail -30 $OUT/peer$pc.log; exit 1; }
grep "^overlap" $OUT/peer$pc.log
done
