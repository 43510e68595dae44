#!/bin/bash
# System-mode bench vs raw bench on the same box (1 GPU).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extras > $OUT/bench_raw.log 2>&1
rc=$?; echo "[raw] rc=$rc"; tail -1 $OUT/bench_raw.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --system --steps 20 --warmup 5 > $OUT/bench_system.log 2>&1
rc=$?; echo "[system] rc=$rc"; tail -2 $OUT/bench_system.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --system --dtype fp16 --steps 20 --warmup 5 > $OUT/bench_system16.log 2>&1
rc=$?; echo "[system fp16] rc=$rc"; tail -1 $OUT/bench_system16.log
exit $rc
