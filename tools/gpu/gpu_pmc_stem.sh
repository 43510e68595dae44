#!/bin/bash
# PMC counters of the fused stem (kernel-trace + pmc only; one pass per counter set).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/pmcs$i -o p -- python3 tools/stem_once.py > $OUT/pmcs$i.log 2>&1
  rc=$?; echo "[pass $i] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmcs*/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "stem_fused" in r.get("Kernel_Name", ""):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    byc = collections.defaultdict(list)
    for (d, c), v in per.items():
        byc[c].append(v)
    for c, v in sorted(byc.items()):
        print(f"{c:28s} {sum(v) / len(v):.4g}  (dispatches={len(v)})")
PY
