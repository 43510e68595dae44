#!/usr/bin/env python3
"""Interleaved per-layer A/B of the fp16 band-staged 3x3 conv (tile 70) against
the im2col fp16 tiles on ResNet50 b1024 / ResNet18 b400 3x3/s1 shapes.

usage: python tools/band_f16_ab.py [--reps 5] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (name, B, H, c, res)
    ("r50 l2", 1024, 28, 128, False), ("r50 l3", 1024, 14, 256, False), ("r50 l4", 1024, 7, 512, False),
    ("r18 l2+res", 400, 28, 128, True), ("r18 l2", 400, 28, 128, False),
    ("r18 l3+res", 400, 14, 256, True), ("r18 l4+res", 400, 7, 512, True),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tiles", default="70,36,42,27")
    a = ap.parse_args()
    from idunno import ops
    from idunno.models.packed import pack_conv_weight

    dev = "cuda"
    tiles = [int(t) for t in a.tiles.split(",")]
    for name, B, H, c, res in SHAPES:
        torch.manual_seed(0)
        w, _ = pack_conv_weight(torch.randn(c, c, 3, 3) / (c * 9) ** 0.5, "fp16")
        w = w.to(dev)
        b = torch.zeros(c, device=dev)
        x = torch.randn(B, H, H, c, device=dev).half()
        r = torch.randn(B, H, H, c, device=dev).half() if res else None
        arms = {f"tile{t}": (lambda t=t: ops.conv2d(x, w, b, 3, 3, 1, 1, True, residual=r, tile=t)) for t in tiles}
        arms["auto-noband"] = lambda: ops.conv2d(x, w, b, 3, 3, 1, 1, True, residual=r, route=1)
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
        flops = 2.0 * B * H * H * c * c * 9
        row = {"layer": name, **{k: round(min(v), 1) for k, v in times.items()}}
        row["band_PF"] = round(flops / row["tile70"] / 1e9, 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
