#!/bin/bash
# PMC counters for selected conv layers (kernel-trace + pmc only; no sys/runtime trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
stop_if_fatal() { local rc=$1; echo "[$2] rc=$rc"; if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then exit "$rc"; fi; }
rocprofv3 -L > $OUT/counters.txt 2>&1; echo "[list] rc=$?"
LAYERS=${LAYERS:-b0c0,b4c1+res}
TILES=${TILES:-15,18,11}
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $OUT/pmc1 -o p1 -- \
  python3 tools/bench_layers.py --batch 400 --rounds 1 --no-stem --layers $LAYERS --tiles $TILES > $OUT/pmc1.log 2>&1
stop_if_fatal $? pmc1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $OUT/pmc2 -o p2 -- \
  python3 tools/bench_layers.py --batch 400 --rounds 1 --no-stem --layers $LAYERS --tiles $TILES > $OUT/pmc2.log 2>&1
stop_if_fatal $? pmc2
echo done
