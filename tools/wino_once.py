#!/usr/bin/env python3
"""Run the fp32 Winograd conv (and the direct conv) a few times at two ResNet18
B=400 layer shapes, for rocprofv3 counter passes (tools/gpu_r2_wino_pmc.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from idunno import ops
    from idunno.models.packed import pack_conv_weight, wino_weight

    ops.load()
    dev = "cuda"
    for (h, c) in ((56, 64), (14, 256)):
        x = torch.randn(400, h, h, c, device=dev)
        w = torch.randn(c, c, 3, 3) / (c * 9) ** 0.5
        b = torch.zeros(c, device=dev)
        u = wino_weight(w).to(dev)
        pw, _ = pack_conv_weight(w, "fp32")
        pw = pw.to(dev)
        for _ in range(3):
            for var in (0, 1, 2):
                ops.conv2d_wino(x, u, b, True, None, var)
            ops.conv2d(x, pw, b, 3, 3, 1, 1, True)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
