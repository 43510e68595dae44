#!/usr/bin/env python3
"""Interleaved A/B of conv_glds plain vs residual variants (and the residual variant
with its residual loads / stores ablated), min over repeats, so clock ramp-up and
run order do not bias one variant.  Profiling only: ablated outputs are wrong."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("l2 28x28 128->128", 28, 128, 128), ("l3 14x14 256->256", 14, 256, 256), ("l4 7x7 512->512", 7, 512, 512)]


def main():
    from idunno import ops
    from idunno.models.packed import pack_conv_weight

    ext = ops.load()
    torch.manual_seed(0)
    B, iters, reps = 400, 50, 7
    cfgs = [("plain", False, 0), ("plain no-stores", False, 1), ("res", True, 0), ("res no-res-loads", True, 2),
            ("res no-stores", True, 1), ("res neither", True, 3)]
    # warm the clocks
    x = torch.randn(B, 28, 28, 128, device="cuda").half()
    w, _ = pack_conv_weight(torch.randn(128, 128, 3, 3) / 34.0)
    w, b = w.cuda(), torch.zeros(128, device="cuda")
    for _ in range(200):
        ops.conv2d(x, w, b, 3, 3, 1, 1, True, None)
    torch.cuda.synchronize()
    for name, H, C, Co in SHAPES:
        x = torch.randn(B, H, H, C, device="cuda").half()
        w, _ = pack_conv_weight(torch.randn(Co, C, 3, 3) / (9 * C) ** 0.5)
        w = w.cuda()
        b = torch.zeros(Co, device="cuda")
        r = torch.randn(B, H, H, Co, device="cuda").half()
        best = {c[0]: 1e9 for c in cfgs}
        for _ in range(reps):
            for cname, has_res, mode in cfgs:
                ext.set_conv_ablation(mode)
                res = r if has_res else None
                ops.conv2d(x, w, b, 3, 3, 1, 1, True, res)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(iters):
                    ops.conv2d(x, w, b, 3, 3, 1, 1, True, res)
                en.record()
                torch.cuda.synchronize()
                best[cname] = min(best[cname], st.elapsed_time(en) / iters * 1e3)
        ext.set_conv_ablation(0)
        for cname, _, _ in cfgs:
            print(f"{name:20s} {cname:18s} {best[cname]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
