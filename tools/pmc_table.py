#!/usr/bin/env python3
"""Per-kernel PMC table from rocprofv3 --pmc csv passes (tools/gpu_pmc_bench.sh).

usage: python tools/pmc_table.py gpurun_out/pmcb1 gpurun_out/pmcb2 ... [--title T]
Counters are summed over dispatches of the same kernel, then turned into:
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 256 CU * 4 SIMD)
               (GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md)
  wait/active= SQ_WAIT_ANY, SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES
  lds_conf   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles share)
  l2_hit     = TCC_HIT / (TCC_HIT + TCC_MISS)
  clk_GHz    = GRBM_GUI_ACTIVE/8 / kernel wall time
"""
import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?idunno::(\w+)(<[^(]*>)?\(", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--title", default="PMC per kernel")
    a = ap.parse_args()
    tot = defaultdict(lambda: defaultdict(float))
    wall = defaultdict(float)
    for d in a.dirs:
        seen = set()
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                key = (r["Dispatch_Id"], k)
                if d == a.dirs[0] and key not in seen:
                    seen.add(key)
                    wall[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    print(f"### {a.title}\n")
    print("| kernel | time ms | clk GHz | mfma_busy | wait | active | lds_conf | lds_wait | l2_hit | TA_busy |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in sorted(tot, key=lambda k: -wall[k]):
        c = tot[k]
        g = c.get("GRBM_GUI_ACTIVE", 0) / 3   # one per pass
        cyc = g / 8 if g else 0
        def share(x, y):
            return f"{x / y:.2f}" if y else "-"
        mb = share(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0), cyc * 256 * 4) if cyc else "-"
        clk = f"{cyc / wall[k] / 1e9:.2f}" if wall[k] and cyc else "-"
        wc = c.get("SQ_WAVE_CYCLES", 0)
        h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        print(f"| `{k}` | {wall[k] * 1e3:.2f} | {clk} | {mb} | {share(c.get('SQ_WAIT_ANY', 0), wc)} | "
              f"{share(c.get('SQ_ACTIVE_INST_ANY', 0), wc)} | "
              f"{share(c.get('SQ_LDS_BANK_CONFLICT', 0), c.get('SQ_LDS_IDX_ACTIVE', 0))} | "
              f"{share(c.get('SQ_WAIT_INST_LDS', 0), wc)} | {share(h, h + m)} | "
              f"{share(c.get('TA_BUSY_avr', 0), cyc) if cyc else '-'} |")


if __name__ == "__main__":
    main()
