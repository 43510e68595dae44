#!/usr/bin/env python3
"""One band-staged split 3x3 conv layer, repeated (for rocprofv3 PMC passes of a
single kernel variant; ``--flags`` selects conv3x3_band.hip ablations).

usage: python tools/band_loop.py --H 28 --c 128 --res --flags 0 --iters 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--H", type=int, default=28)
    ap.add_argument("--c", type=int, default=128)
    ap.add_argument("--res", action="store_true")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models.packed import pack_split_weight

    ext = ops.load()
    dev = "cuda"
    torch.manual_seed(0)
    sw, scale = pack_split_weight(torch.randn(a.c, a.c, 3, 3) / (a.c * 9) ** 0.5)
    sw = sw.to(dev)
    b = torch.zeros(a.c, device=dev)
    xs = ops.split_from_f32(torch.randn(a.batch, a.H, a.H, a.c, device=dev))
    rs = ops.split_from_f32(torch.randn(a.batch, a.H, a.H, a.c, device=dev)) if a.res else None
    for _ in range(a.iters):
        ext.conv3x3_band_split(xs, sw, b, rs, True, scale, False, 0, a.flags)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
