#!/usr/bin/env python3
"""Ablation of the fp32 Winograd kernel (8-wave variant) at two ResNet18 B=400
shapes: time with the DMA / raw read+transform / U reads / epilogue stores
removed (results wrong; set_wino_ablation is profiling-only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
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
    dev = "cuda"
    modes = [(0, "full"), (1, "no DMA"), (2, "no raw/transform"), (4, "no U reads"), (8, "no stores"),
             (6, "no LDS reads"), (7, "MFMA + stores only"), (15, "MFMA only"), (16 | 1, "setup + epilogue only")]
    print("| shape | variant | " + " | ".join(n for _, n in modes) + " |")
    print("|---|---|" + "---:|" * len(modes))
    for (h, c) in ((56, 64), (28, 128), (14, 256), (7, 512)):
        x = torch.randn(400, h, h, c, device=dev)
        w = torch.randn(c, c, 3, 3) / (c * 9) ** 0.5
        b = torch.zeros(c, device=dev)
        u = wino_weight(w).to(dev)
        for var in (1, 3):
            for pair in (False,):
                C.set_wino_pairing(pair)
                row = []
                for m, _ in modes:
                    C.set_wino_ablation(m)
                    row.append(timeit(lambda: ops.conv2d_wino(x, u, b, True, None, var)))
                C.set_wino_ablation(0)
                print(f"| {h}x{h}x{c} | {({1: '8w', 3: '4w x2/CU', 0: '4w', 2: '4w pipe'})[var]}{' pair' if pair else ''} | "
                      + " | ".join(f"{t:.0f}" for t in row) + " |", flush=True)
        C.set_wino_pairing(False)


if __name__ == "__main__":
    main()
