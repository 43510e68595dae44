#!/usr/bin/env python3
"""Interleaved A/B of the band-staged split 3x3 conv (tile 70, flag variants)
against the im2col split tiles on ResNet18 layer shapes at B = 400.

usage: python tools/band_ab.py [--batch 400] [--reps 5] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (name, H, cin, cout, res)
    ("l2 c1+res", 28, 128, 128, True), ("l2 c0", 28, 128, 128, False),
    ("l3 c1+res", 14, 256, 256, True), ("l3 c0", 14, 256, 256, False),
    ("l4 c1+res", 7, 512, 512, True), ("l4 c0", 7, 512, 512, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--flags", default="0,2,4,6", help="conv3x3_band.hip profiling ablations: 2 no stores, 4 no residual loads")
    ap.add_argument("--tiles", default="36,42")
    a = ap.parse_args()
    from idunno import ops
    from idunno.models.packed import pack_split_weight

    ext = ops.load()
    dev = "cuda"
    flags = [int(f) for f in a.flags.split(",")]
    tiles = [int(t) for t in a.tiles.split(",")]
    out = []
    for name, H, cin, cout, res in SHAPES:
        torch.manual_seed(0)
        w = torch.randn(cout, cin, 3, 3) / (cin * 9) ** 0.5
        sw, scale = pack_split_weight(w)
        sw = sw.to(dev)
        b = torch.zeros(cout, device=dev)
        xs = ops.split_from_f32(torch.randn(a.batch, H, H, cin, device=dev))
        rs = ops.split_from_f32(torch.randn(a.batch, H, H, cout, device=dev)) if res else None
        arms = {f"tile{t}": (lambda t=t: ops.conv2d_split(xs, sw, b, scale, 3, 3, 1, 1, True, residual=rs, tile=t))
                for t in tiles}
        for f in flags:
            arms[f"band f{f}"] = lambda f=f: ext.conv3x3_band_split(xs, sw, b, rs, True, scale, False, 0, f)
        times = {k: [] for k in arms}
        for _ in range(a.reps):
            for k, fn in arms.items():
                fn()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(a.iters):
                    fn()
                en.record()
                torch.cuda.synchronize()
                times[k].append(st.elapsed_time(en) * 1000 / a.iters)
        flops = 2.0 * a.batch * H * H * cout * cin * 9 * 3     # f16 MFMA work (3 products per split MAC)
        row = {"layer": name, **{k: round(min(v), 1) for k, v in times.items()}}
        best = min(row[k] for k in times)
        row["best_PF"] = round(flops / best / 1e9, 3)
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
