#!/bin/bash
# PMC passes over the fused AlexNet stem variants (tools/astem_ablate.py), one
# rocprofv3 run per counter pass, then the per-kernel table.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_astem; mkdir -p $OUT; export TMPDIR=/tmp
V=${1:-64,65,66}
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P3="SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM TA_BUSY_avr GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$i -o p -- \
    python3 tools/astem_ablate.py 500 $V > $OUT/p$i.log 2>&1
  rc=$?; echo "[pmc$i] rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
echo done
