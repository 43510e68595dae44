#!/usr/bin/env python3
"""Summarise rocprofv3 kernel statistics into a markdown table.

usage: python tools/prof_summary.py <kernel_stats.csv | results.db> [--per N] [--title T]
  input     a ``--stats --output-format csv`` kernel_stats.csv, or the default
            rocpd SQLite database (``<name>_results.db``) written by rocprofv3
  --per N   divide totals by N (e.g. number of forwards) to get per-step time
"""
import argparse
import csv
import re
import sqlite3


def short(name: str) -> str:
    m = re.match(r"void idunno::(\w+)<(.*)>\(", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.match(r"(?:void )?idunno::(\w+)\(", name)
    if m:
        return m.group(1)
    m = re.match(r"_ZN6idunno\d+(\w+?)E", name)
    if m:
        return m.group(1)
    return name[:80]


def rows_csv(path):
    for r in csv.DictReader(open(path)):
        yield r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]), None


def rows_db(path):
    c = sqlite3.connect(path)
    res = {}
    for name, n, tot, vgpr, agpr, lds in c.execute(
            "select name, count(*), sum(duration), max(vgpr_count), max(accum_vgpr_count), max(lds_size) "
            "from kernels group by name order by sum(duration) desc"):
        res[name] = (n, float(tot), f"{vgpr}/{agpr}/{lds // 1024 if lds else 0}K")
    for name, (n, tot, res_s) in res.items():
        yield name, n, tot, tot / n, res_s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--title", default="kernel stats")
    a = ap.parse_args()
    rows = list(rows_db(a.path) if a.path.endswith(".db") else rows_csv(a.path))
    tot = sum(r[2] for r in rows)
    res_col = any(r[4] for r in rows)
    print(f"### {a.title}\n")
    print("| kernel | calls | avg us | total ms | per-step us | % |" + (" vgpr/agpr/lds |" if res_col else ""))
    print("|---|---:|---:|---:|---:|---:|" + ("---|" if res_col else ""))
    for name, n, t, avg, res_s in rows:
        line = f"| `{short(name)}` | {n} | {avg / 1e3:.1f} | {t / 1e6:.3f} | {t / 1e3 / a.per:.1f} | {100 * t / tot:.1f} |"
        print(line + (f" {res_s} |" if res_col else ""))
    print(f"\nsum of kernel time: {tot / 1e6:.3f} ms ({tot / 1e3 / a.per:.1f} us per step)")


if __name__ == "__main__":
    main()
