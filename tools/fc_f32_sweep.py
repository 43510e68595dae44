#!/usr/bin/env python3
"""fp32 FC layers (1x1 conv on a 1x1 image) at the models' batch sizes: every
conv_f32 tile id vs the default pick (profiles/r2_v16_fc_f32_sweep.md)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wino_variants import timeit  # noqa: E402


def main():
    from idunno import ops

    C = ops.load()
    shapes = [(500, 9216, 4096), (500, 4096, 4096), (500, 4096, 1000), (400, 512, 1000), (1024, 2048, 1000)]
    tiles = [-1] + [t for t in range(100, 110)]
    print("| M x K -> N | default | " + " | ".join(str(t) for t in tiles[1:]) + " |")
    print("|---|" + "---:|" * len(tiles))
    for (m, k, n) in shapes:
        x = torch.randn(m, 1, 1, k, device="cuda")
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.zeros(n, device="cuda")
        row = []
        for t in tiles:
            try:
                row.append(f"{timeit(lambda: C.conv2d_nhwc_f32(x, w, b, None, 1, 1, 1, 0, True, t, None)):.0f}")
            except RuntimeError:
                row.append("-")
        print(f"| {m} x {k} -> {n} | " + " | ".join(row) + " |", flush=True)
    print()
    print("split-K in one launch (linear_f32_splitk), tiles 103 / 107 / default:")
    print()
    print("| M x K -> N | splits | 103 | 107 | default | max rel err |")
    print("|---|---:|---:|---:|---:|---:|")
    for (m, k, n) in shapes:
        x = torch.randn(m, k, device="cuda")
        w = torch.randn(n, k, device="cuda") / k ** 0.5
        b = torch.randn(n, device="cuda")
        ref = torch.relu(x.double() @ w.double().t() + b.double())
        for sp in (1, 2, 4, 8):
            if k % (16 * sp):
                continue
            row = [f"{timeit(lambda: C.linear_f32_splitk(x, w, b, True, sp, t)):.0f}" for t in (103, 107, -1)]
            err = ((C.linear_f32_splitk(x, w, b, True, sp, -1).double() - ref).abs().max() / ref.abs().max()).item()
            print(f"| {m} x {k} -> {n} | {sp} | " + " | ".join(row) + f" | {err:.1e} |", flush=True)


if __name__ == "__main__":
    main()
