#!/usr/bin/env python3
"""Per-conv time of one eager forward against its HBM and MFMA rooflines.

Every conv launch of the HipRunner forward (fp16 or the split fp32 path) is
bracketed by events (eager, one launch at a time, after a warm-up forward),
and reported with its minimum HBM traffic (input once, residual, output; no
im2col re-reads) and its FLOPs, so the memory-bound layers stand out.

usage: python tools/layer_roofline.py [--model resnet50] [--batch 1024] [--dtype fp16]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM_TBS = 6.0            # achievable HBM3E (MICROARCH: ~6.3 TB/s)
MFMA_F16_TFS = 2200.0    # dense f16 at the ~2.1 GHz the chip holds under MFMA load


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program

    ops.load()
    dev = "cuda"
    prog = build_program(a.model, dtype=a.dtype)
    runner = HipRunner(prog, dev)
    img = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device=dev)
    runner.logits(img)
    torch.cuda.synchronize()

    recs = []
    names = ("conv2d", "conv2d_split", "stem_fused", "stem_split", "linear", "linear_split", "global_avgpool",
             "conv3x3_c64", "conv1x1_dual", "conv1x1_dual_split", "conv1x1_fused_next")
    orig = {n: getattr(ops, n) for n in names if hasattr(ops, n)}

    def wrap(n, f):
        def g(*args, **kw):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = f(*args, **kw)
            e1.record()
            y = out[0] if isinstance(out, tuple) else out    # conv1x1_fused_next: (y, z)
            x = args[0]
            res = kw.get("residual")
            recs.append((n, tuple(x.shape), x.element_size(), tuple(y.shape), y.element_size(),
                         None if res is None else res.numel() * res.element_size(), args, e0, e1))
            return out
        return g

    per = collections.defaultdict(list)
    for r in range(a.reps):
        recs.clear()
        for n, f in orig.items():
            setattr(ops, n, wrap(n, f))
        try:
            runner.logits(img)
        finally:
            for n, f in orig.items():
                setattr(ops, n, f)
        torch.cuda.synchronize()
        for i, (n, xs, xe, ys, ye, rb, args, e0, e1) in enumerate(recs):
            per[i].append(e0.elapsed_time(e1) * 1e3)
    print(f"### {a.model} B={a.batch} {a.dtype}: per-launch time vs rooflines (eager, median of {a.reps})\n")
    print("| # | op | in | out | us | min HBM MB | GB/s | % HBM | GFLOP | TF/s |")
    print("|---:|---|---|---|---:|---:|---:|---:|---:|---:|")
    tot = collections.Counter()
    for i, (n, xs, xe, ys, ye, rb, args, e0, e1) in enumerate(recs):
        us = sorted(per[i])[len(per[i]) // 2]
        nbytes = (torch.Size(xs).numel() * xe + torch.Size(ys).numel() * ye + (rb or 0))
        gflop = 0.0
        if n in ("conv2d", "conv2d_split") and len(ys) == 4:
            # N from the weights (rows = output channels), not from the output tensor: a
            # split output carries 2 halfs per channel, an fp32 (OUT_F32) one 1 float --
            # halving the last dim miscounted the f32-output split conv
            w = args[1]
            k = w.shape[1] if n == "conv2d" else w.shape[1] // 2
            gflop = 2.0 * torch.Size(ys[:3]).numel() * w.shape[0] * k / 1e9
        gbs = nbytes / (us * 1e-6) / 1e9
        tf = gflop / (us * 1e-6) / 1e3 if gflop else 0.0
        kind = n + ("+res" if rb else "")
        tot[kind] += us
        tot["all"] += us
        print(f"| {i} | {kind} | {list(xs)} | {list(ys)} | {us:.0f} | {nbytes / 1e6:.0f} | {gbs:.0f} | "
              f"{100 * gbs / (HBM_TBS * 1e3):.0f} | {gflop:.1f} | {tf:.0f} |")
    print()
    for k, v in tot.most_common():
        print(f"- {k}: {v / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
