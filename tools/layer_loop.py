#!/usr/bin/env python3
"""Run one split conv layer shape repeatedly through the given tile ids (for
rocprofv3 kernel traces / PMC passes of single kernels).

usage: python tools/layer_loop.py --H 28 --cin 128 --cout 128 --res --tiles 36,70 --iters 20
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
    ap.add_argument("--cin", type=int, default=128)
    ap.add_argument("--cout", type=int, default=128)
    ap.add_argument("--res", action="store_true")
    ap.add_argument("--tiles", default="36,70")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models.packed import pack_split_weight

    ops.load()
    dev = "cuda"
    torch.manual_seed(0)
    w = torch.randn(a.cout, a.cin, 3, 3) / (a.cin * 9) ** 0.5
    sw, scale = pack_split_weight(w)
    sw = sw.to(dev)
    b = torch.zeros(a.cout, device=dev)
    xs = ops.split_from_f32(torch.randn(a.batch, a.H, a.H, a.cin, device=dev))
    rs = ops.split_from_f32(torch.randn(a.batch, a.H, a.H, a.cout, device=dev)) if a.res else None
    tiles = [int(t) for t in a.tiles.split(",")]
    for _ in range(a.iters):
        for t in tiles:
            ops.conv2d_split(xs, sw, b, scale, 3, 3, 1, 1, True, residual=rs, tile=t)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
