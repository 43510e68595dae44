#!/usr/bin/env python3
"""Same-box A/B: Winograd variant 3 with e-GEMMs one at a time vs in pairs
(set_wino_pairing), best of 3 alternating rounds, ResNet18 B=400 shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wino_variants import timeit  # noqa: E402


def main():
    from idunno import ops
    from idunno.models.packed import wino_weight

    C = ops.load()
    print("| shape | single e | e pairs | pairs/single |")
    print("|---|---:|---:|---:|")
    for (h, ch) in ((56, 64), (28, 128), (14, 256), (7, 512)):
        x = torch.randn(400, h, h, ch, device="cuda")
        w = torch.randn(ch, ch, 3, 3) / (ch * 9) ** 0.5
        b = torch.zeros(ch, device="cuda")
        u = wino_weight(w).to("cuda")
        t = {False: 1e9, True: 1e9}
        for _ in range(3):
            for pair in (False, True):
                C.set_wino_pairing(pair)
                t[pair] = min(t[pair], timeit(lambda: ops.conv2d_wino(x, u, b, True, None, 3)))
        C.set_wino_pairing(False)
        print(f"| {h}x{h}x{ch} | {t[False]:.0f} | {t[True]:.0f} | {t[True] / t[False]:.3f} |", flush=True)


if __name__ == "__main__":
    main()
