#!/bin/bash
# PMC passes over the band-staged split 3x3 conv (tools/band_loop.py), one
# rocprofv3 run per (flags, pass):  tools/gpu/pmc_band.sh TAG "<band_loop args>" FLAGS...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:?tag}; ARGS=${2:-}; shift 2
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for F in "$@"; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/f$F/p$i -o p -- \
      python3 tools/band_loop.py $ARGS --flags $F > $OUT/f${F}_p$i.log 2>&1
    rc=$?; echo "[f$F pmc$i] rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/f${F}_p$i.log; exit $rc; fi
  done
  python3 tools/pmc_table.py $OUT/f$F/p1 $OUT/f$F/p2 $OUT/f$F/p3 --title "$TAG flags $F" > $OUT/table_f$F.md
done
echo done
