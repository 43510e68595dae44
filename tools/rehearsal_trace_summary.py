#!/usr/bin/env python3
"""Summarise a multi-process rocprofv3 kernel trace of the N-rank rehearsal
(``tools/rehearse_n8.sh ... prof``: one ``<pid>_kernel_trace.csv`` per rank
process, all on the same GPU) as markdown.

Per rank: forward kernels (everything that is not RCCL) and RCCL kernels --
count, total, mean and max duration, and the share of the rank's busy time the
RCCL kernels take.  Over all ranks, inside the window where every rank ran its
forwards (the last ``--tail`` forwards of each rank): the share of wall time in
which at least one forward kernel ran (GPU compute) and in which only RCCL
kernels ran (every rank waiting on a collective).

    python tools/rehearsal_trace_summary.py gpurun_out/TAG/prof > profiles/x.md
"""
from __future__ import annotations

import argparse
import csv
import glob
import os


def _load(path: str) -> list[tuple[int, int, str]]:
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    out.sort()
    return out


def _union(iv: list[tuple[int, int]]) -> int:
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def _is_rccl(name: str) -> bool:
    return "rccl" in name.lower() or "nccl" in name.lower()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--fwd-kernel", default="softmax_top1", help="kernel that ends one forward")
    ap.add_argument("--tail", type=int, default=10, help="forwards per rank in the analysed window")
    a = ap.parse_args()
    ranks = {}
    for p in sorted(glob.glob(os.path.join(a.dir, "*_kernel_trace.csv"))):
        k = _load(p)
        if any(a.fwd_kernel in n for _, _, n in k):
            ranks[os.path.basename(p).split("_")[0]] = k
    if not ranks:
        raise SystemExit("no rank traces with forwards")
    # window: from the earliest start of the last `tail` forwards of any rank to the latest end
    ends = {pid: [e for _, e, n in k if a.fwd_kernel in n] for pid, k in ranks.items()}
    n_fwd = min(len(v) for v in ends.values())
    tail = min(a.tail, n_fwd - 1)
    w0 = min(v[-tail - 1] for v in ends.values())
    w1 = max(v[-1] for v in ends.values())
    print(f"# Rehearsal kernel trace: {len(ranks)} rank processes on one GPU\n")
    print(f"Source: `{a.dir}` (rocprofv3 --kernel-trace, one file per process). Window: the last {tail} "
          f"forwards of every rank, {(w1 - w0) / 1e6:.1f} ms.\n")
    print("| rank pid | forward kernels | forward ms | RCCL kernels | RCCL ms | RCCL mean ms | RCCL max ms "
          "| RCCL share of rank's kernel time |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    fwd_iv, rccl_iv = [], []
    for pid, k in ranks.items():
        win = [(max(s, w0), min(e, w1), n) for s, e, n in k if e > w0 and s < w1]
        f = [(s, e) for s, e, n in win if not _is_rccl(n)]
        r = [(s, e) for s, e, n in win if _is_rccl(n)]
        fwd_iv += f
        rccl_iv += r
        ft, rt = sum(e - s for s, e in f) / 1e6, sum(e - s for s, e in r) / 1e6
        rmean = rt / len(r) if r else 0.0
        rmax = max((e - s for s, e in r), default=0) / 1e6
        share = rt / (ft + rt) if ft + rt else 0.0
        print(f"| {pid} | {len(f)} | {ft:.1f} | {len(r)} | {rt:.1f} | {rmean:.2f} | {rmax:.1f} | {share:.2f} |")
    wall = w1 - w0
    busy_fwd = _union(fwd_iv)
    busy_any = _union(fwd_iv + rccl_iv)
    print()
    print(f"- wall time with at least one forward kernel running (any rank): **{busy_fwd / wall:.2f}**")
    print(f"- wall time with only RCCL kernels running (every rank in a collective): "
          f"**{(busy_any - busy_fwd) / wall:.2f}**")
    print(f"- wall time with no kernel at all: {(wall - busy_any) / wall:.2f}")


if __name__ == "__main__":
    main()
