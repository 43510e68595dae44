#!/usr/bin/env python3
"""How much of a conv_glds layer is its epilogue?  Times ResNet layer shapes with
the epilogue stores and/or residual loads ablated (profiling only: ablated
outputs are wrong)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("l2 28x28 128->128", 28, 128, 128), ("l3 14x14 256->256", 14, 256, 256), ("l4 7x7 512->512", 7, 512, 512)]
# ResNet50 1x1 convs at B = 1024 (--r50): the memory-bound bottleneck layers
SHAPES_R50 = [("r50 l1 56x56 64->256", 56, 64, 256), ("r50 l1 56x56 256->64", 56, 256, 64),
              ("r50 l2 28x28 128->512", 28, 128, 512), ("r50 l3 14x14 256->1024", 14, 256, 1024),
              ("r50 l4 7x7 512->2048", 7, 512, 2048)]


def main():
    from idunno import ops
    from idunno.models.packed import pack_conv_weight

    ext = ops.load()
    torch.manual_seed(0)
    r50 = "--r50" in sys.argv
    B = 1024 if r50 else 400
    k = 1 if r50 else 3
    modes = {0: "full", 1: "no stores", 2: "no residual loads", 3: "neither"}
    for name, H, C, Co in (SHAPES_R50 if r50 else SHAPES):
        x = torch.randn(B, H, H, C, device="cuda").half()
        w, _ = pack_conv_weight(torch.randn(Co, C, k, k) / (k * k * C) ** 0.5)
        w = w.cuda()
        b = torch.zeros(Co, device="cuda")
        r = torch.randn(B, H, H, Co, device="cuda").half()
        for res in (None, r):
            for mode, mname in modes.items():
                if res is None and mode & 2:
                    continue
                ext.set_conv_ablation(mode)
                ops.conv2d(x, w, b, k, k, 1, k // 2, True, res)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(20):
                    ops.conv2d(x, w, b, k, k, 1, k // 2, True, res)
                en.record()
                torch.cuda.synchronize()
                print(f"{name:20s} {'res' if res is not None else '   '} {mname:18s} "
                      f"{st.elapsed_time(en) / 20 * 1e3:7.1f} us", flush=True)
    ext.set_conv_ablation(0)


if __name__ == "__main__":
    main()
