#!/bin/bash
# One GPU session: build check, GPU tests, bench, rocprof kernel stats.
# Any fault/abort/timeout (exit >= 124, or 134/139) ends the script at once.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = rc, $2 = step
  local rc=$1
  echo "[$2] rc=$rc"
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
    echo "fatal rc in $2, stopping"; exit "$rc"
  fi
}
python -c "import idunno, idunno._C; print('import ok', idunno.__file__)" > $OUT/import.log 2>&1
stop_if_fatal $? import
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
stop_if_fatal $? pytest_gpu
tail -5 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup ${WARMUP:-5} > $OUT/bench.log 2>&1
stop_if_fatal $? bench
tail -2 $OUT/bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
      python3 bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1
  stop_if_fatal $? rocprof
fi
echo done
