#!/usr/bin/env python3
"""fp16 FC layers: one-launch split-K (linear_splitk) at the models' batch sizes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wino_variants import timeit  # noqa: E402


def main():
    from idunno import ops

    C = ops.load()
    shapes = [(500, 9216, 4096), (500, 4096, 4096), (500, 4096, 1000), (400, 512, 1000), (1024, 2048, 1000)]
    print("| M x K -> N | unsplit | 2 | 4 | 8 | max rel err (4) |")
    print("|---|---:|---:|---:|---:|---:|")
    for (m, k, n) in shapes:
        x = torch.randn(m, k, device="cuda").half()
        w = (torch.randn(n, k, device="cuda") / k ** 0.5).half()
        b = torch.randn(n, device="cuda")
        row = [f"{timeit(lambda: ops.linear(x, w, b, True, True, 1)):.0f}"]
        for sp in (2, 4, 8):
            row.append(f"{timeit(lambda: C.linear_splitk(x, w, b, True, True, sp, -1)):.0f}" if k % (64 * sp) == 0 else "-")
        ref = torch.relu(x.double() @ w.double().t() + b.double())
        y = C.linear_splitk(x, w, b, True, True, 4, -1) if k % 256 == 0 else ops.linear(x, w, b, True, True, 1)
        err = ((y.double() - ref).abs().max() / ref.abs().max()).item()
        print(f"| {m} x {k} -> {n} | " + " | ".join(row) + f" | {err:.1e} |", flush=True)


if __name__ == "__main__":
    main()
