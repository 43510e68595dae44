#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv into a markdown table.

usage: python tools/prof_summary.py <kernel_stats.csv> [--per N] [--title T]
  --per N   divide totals by N (e.g. number of forwards) to get per-step time
"""
import argparse
import csv
import re


def short(name: str) -> str:
    m = re.match(r"void idunno::(\w+)<(.*)>\(", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.match(r"_ZN6idunno\d+(\w+?)E", name)
    if m:
        return m.group(1)
    return name[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--title", default="kernel stats")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"### {a.title}\n")
    print(f"| kernel | calls | avg us | total ms | per-step us | % |")
    print("|---|---:|---:|---:|---:|---:|")
    for r in rows:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {t/1e6:.3f} | "
              f"{t/1e3/a.per:.1f} | {100*t/tot:.1f} |")
    print(f"\nsum of kernel time: {tot/1e6:.3f} ms ({tot/1e3/a.per:.1f} us per step)")


if __name__ == "__main__":
    main()
