#!/bin/bash
# why the raw headline loop collapses in the 8-rank RCCL
# rehearsal on ONE GPU (8 processes share the card) while the runtime path holds.
#   tools/rehearse_n8.sh TAG [variants...]
# variants: q4 (HIP default queues), spin (--host-wait spin), q1 (GPU_MAX_HW_QUEUES=1), n4, prof (rocprofv3
# kernel trace of the 8-rank headline).  Each step has its own limit; stop at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:?tag}; shift
STEPS=${*:-q4 q1 n4 prof}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--rehearse-rccl --no-system --no-extras --steps 20 --warmup 5 --launch-timeout 240"
for s in $STEPS; do
  case $s in
    q4) timeout -k 10 300 python -u bench.py --gpus 8 $ARGS --json-out $OUT/n8_q4.json > $OUT/n8_q4.log 2>&1 || exit 11 ;;
    hwq4) IDUNNO_REHEARSE_HW_QUEUES=4 timeout -k 10 300 python -u bench.py --gpus 8 $ARGS --json-out $OUT/n8_hwq4.json \
          > $OUT/n8_hwq4.log 2>&1 || exit 18 ;;
    full) timeout -k 10 900 python -u bench.py --gpus 8 --rehearse-rccl --steps 20 --warmup 5 \
          --json-out $OUT/n8_full.json > $OUT/n8_full.log 2>&1 || exit 19 ;;
    spin) timeout -k 10 300 python -u bench.py --gpus 8 $ARGS --host-wait spin --json-out $OUT/n8_spin.json \
          > $OUT/n8_spin.log 2>&1 || exit 17 ;;
    q1) GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python -u bench.py --gpus 8 $ARGS --json-out $OUT/n8_q1.json \
          > $OUT/n8_q1.log 2>&1 || exit 12 ;;
    q2) GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -u bench.py --gpus 8 $ARGS --json-out $OUT/n8_q2.json \
          > $OUT/n8_q2.log 2>&1 || exit 12 ;;
    nopipe) timeout -k 10 300 python -u bench.py --gpus 8 $ARGS --no-pipeline --json-out $OUT/n8_nopipe.json \
          > $OUT/n8_nopipe.log 2>&1 || exit 15 ;;
    n4) timeout -k 10 300 python -u bench.py --gpus 4 $ARGS --json-out $OUT/n4_q4.json > $OUT/n4_q4.log 2>&1 || exit 13 ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o %pid% -- \
            python -u bench.py --gpus 8 --rehearse-rccl --no-system --no-extras --steps 10 --warmup 3 \
            --launch-timeout 240 > $OUT/prof.log 2>&1 || exit 14 ;;
    sys8) timeout -k 10 400 python -u bench.py --gpus 8 --rehearse-rccl --system --steps 20 --warmup 5 \
            --two-job-queries 4 --sdfs-images 0 --ref-delay-queries 0 --extras-timeout 300 \
            --json-out $OUT/n8_system.json > $OUT/n8_system.log 2>&1 || exit 16 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
