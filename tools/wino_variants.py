#!/usr/bin/env python3
"""Same-box A/B of fp32 Winograd kernel variants at the ResNet18 B=400 3x3
shapes (best of 3 alternating rounds): usage wino_variants.py 3 5"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) * 1000 / iters


def main():
    from idunno import ops
    from idunno.models.packed import wino_weight

    vs = [int(v) for v in sys.argv[1:]] or [3, 5]
    print("| shape | " + " | ".join(f"v{v} us" for v in vs) + " | rel err (last) |")
    print("|---|" + "---:|" * (len(vs) + 1))
    for (h, ch) in ((56, 64), (28, 128), (14, 256), (7, 512)):
        x = torch.randn(400, h, h, ch, device="cuda")
        w = torch.randn(ch, ch, 3, 3) / (ch * 9) ** 0.5
        b = torch.zeros(ch, device="cuda")
        r = torch.randn(400, h, h, ch, device="cuda")
        u = wino_weight(w).to("cuda")
        t = {v: 1e9 for v in vs}
        for _ in range(3):
            for v in vs:
                t[v] = min(t[v], timeit(lambda: ops.conv2d_wino(x, u, b, True, r, v)))
        y = ops.conv2d_wino(x, u, b, True, r, vs[-1])
        ref = torch.relu(torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.cuda(), b, padding=1)
                         + r.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        print(f"| {h}x{h}x{ch} | " + " | ".join(f"{t[v]:.0f}" for v in vs) + f" | {err:.1e} |", flush=True)
        del x, r, y, ref


if __name__ == "__main__":
    main()
