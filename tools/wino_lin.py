#!/usr/bin/env python3
"""A/B of the variant-3 Winograd blocking at the ResNet18 B=400 shapes:
consecutive-tile (LIN) blocks vs rectangular tile-row / whole-image blocks,
same process, same box (profiles/r2_v8_wino_linear.md)."""
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

    C = ops.load()
    cfgs = [(False, False), (True, False), (True, True)]
    print("| shape | rect us | LIN us | LIN + rotated rows us | best/rect | max rel err (default vs direct) |")
    print("|---|---:|---:|---:|---:|---:|")
    for (h, ch) in ((56, 64), (28, 128), (14, 256), (7, 512)):
        c = ch
        x = torch.randn(400, h, h, c, device="cuda")
        w = torch.randn(c, c, 3, 3) / (c * 9) ** 0.5
        b = torch.zeros(c, device="cuda")
        u = wino_weight(w).to("cuda")
        t = {c: 1e9 for c in cfgs}
        for _ in range(3):            # alternate, keep the best of 3 (clock ramp / order effects)
            for c in cfgs:
                C.set_wino_linear(c[0])
                C.set_wino_rotation(c[1])
                t[c] = min(t[c], timeit(lambda: ops.conv2d_wino(x, u, b, True, None, 3)))
        C.set_wino_linear(True)
        C.set_wino_rotation(False)
        y = ops.conv2d_wino(x, u, b, True, None, 3)
        ref = torch.relu(torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.cuda(), b, padding=1)).permute(0, 2, 3, 1)
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        r = [t[c] for c in cfgs]
        print(f"| {h}x{h}x{ch} | {r[0]:.0f} | {r[1]:.0f} | {r[2]:.0f} | {min(r) / r[0]:.3f} | {err:.1e} |", flush=True)
        del x, y, ref


if __name__ == "__main__":
    main()
