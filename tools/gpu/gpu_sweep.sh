#!/bin/bash
# conv tile sweep only (no torch reference), plus bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "tiles or stem or runner" > $OUT/pytest_tiles.log 2>&1
stop_if_fatal $? pytest_tiles
tail -2 $OUT/pytest_tiles.log
timeout -k 10 600 python tools/bench_layers.py --batch 400 --rounds 2 --tiles ${TILES:-auto,1,11,13,15,16,18,20,23,24,25,26,27,28,29,30,31} --json $OUT/sweep.json > $OUT/sweep.log 2>&1
stop_if_fatal $? sweep
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1
stop_if_fatal $? bench
tail -1 $OUT/bench.log
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $OUT/pmcb -o b -- \
  python3 bench.py --steps 3 --warmup 2 > $OUT/pmcb.log 2>&1
stop_if_fatal $? pmc_bench
echo done
