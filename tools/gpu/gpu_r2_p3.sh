#!/bin/bash
# Packed-row fp32 stems: tests, bench, kernel table.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/p3; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_f32_gpu.py \
    -k "pack3 or model or runner or small_c" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python -u tools/stem_pack3_sweep.py > $OUT/sweep.md 2>&1 || { echo "sweep failed"; tail -20 $OUT/sweep.md; exit 1; }
cat $OUT/sweep.md
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-extras > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof.log; exit 1; }
timeout -k 10 300 python -u bench.py --model alexnet --batch 500 --steps 20 --warmup 5 --no-extras > $OUT/alex.log 2>&1 || { echo "alex failed"; tail -20 $OUT/alex.log; exit 1; }
tail -1 $OUT/alex.log | cut -c1-300
