#!/bin/bash
# PMC passes over the ResNet50 b1024 fp16 forward (single process: tools/fwd_loop.py)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/pmc_r50; mkdir -p $OUT; export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$i -o p -- \
    python3 tools/fwd_loop.py --model resnet50 --batch 1024 --dtype fp16 --iters 3 > $OUT/p$i.log 2>&1
  rc=$?; echo "[pmc$i] rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
echo done
