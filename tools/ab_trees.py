#!/usr/bin/env python3
"""Same-box A/B of two source trees (each with its own built idunno/_C.so):
alternating processes, each timing hipGraph replays of the whole forward
(cdna_hip_programming §5.4 rule 24: interleave, never compare across boxes).

usage: python tools/ab_trees.py TREE_A TREE_B [--rounds 5] [--dtype fp32] [--batch 400] [--model resnet18]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

CHILD = r'''
import sys, time, json, torch
sys.path.insert(0, ".")
from idunno import ops
from idunno.models import HipRunner, build_program
dev = torch.device("cuda")
r = HipRunner(build_program(MODEL, dtype=DTYPE), dev)
shard = ops.synth_images(1234, 0, BATCH, dev)
_s, run = r.capture_window(shard, BATCH)
for _ in range(10):
    run()
torch.cuda.synchronize()
best = []
for _ in range(3):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(ITERS):
        run()
    en.record()
    torch.cuda.synchronize()
    best.append(st.elapsed_time(en) / ITERS)
print(json.dumps({"ms": min(best)}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trees", nargs=2)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    code = (CHILD.replace("MODEL", repr(a.model)).replace("DTYPE", repr(a.dtype))
            .replace("BATCH", str(a.batch)).replace("ITERS", str(a.iters)))
    res = {t: [] for t in a.trees}
    for _ in range(a.rounds):
        for t in a.trees:
            out = subprocess.run([sys.executable, "-c", code], cwd=t, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(out.returncode)
            ms = json.loads(out.stdout.strip().splitlines()[-1])["ms"]
            res[t].append(ms)
            print(f"{a.model} b{a.batch} {a.dtype} {os.path.basename(os.path.abspath(t))}: {ms:.4f} ms", flush=True)
    med = {t: statistics.median(v) for t, v in res.items()}
    ta, tb = a.trees
    print(f"median {ta}: {med[ta]:.4f} ms  {tb}: {med[tb]:.4f} ms  B vs A: {100 * (med[ta] / med[tb] - 1):+.2f}% throughput")


if __name__ == "__main__":
    main()
