#!/bin/bash
# PMC passes over the whole ResNet18 b400 forward (tools/fwd_loop.py), one
# rocprofv3 run per pass, then the per-kernel table (tools/pmc_table.py).
#   tools/gpu/pmc_forward.sh TAG "<fwd_loop args>"
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}; ARGS=${2:-}
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$i -o p -- \
    python3 tools/fwd_loop.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "[pmc$i] rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_table.py $OUT/p1 $OUT/p2 $OUT/p3 --title "$TAG" > $OUT/table.md
echo done
