#!/usr/bin/env python3
"""fp32 RGB stems at B=400 (ResNet 7x7/2) / 500 (AlexNet 11x11/4): NHWC4 small-C
path vs packed rows, every tile id, plus the two preprocess kernels."""
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
    from idunno.models.packed import pack_conv_weight, pack_conv_weight_p3

    ops.load()
    for (B, k, s, p) in ((400, 7, 2, 3), (500, 11, 4, 2)):
        img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
        w = torch.randn(64, 3, k, k) / (3 * k * k) ** 0.5
        b = torch.zeros(64, device="cuda")
        w4 = pack_conv_weight(w, "fp32")[0].cuda()
        w3 = pack_conv_weight_p3(w).cuda()
        x4 = ops.preprocess(img, f32=True)
        x3 = ops.preprocess_pack3(img, k, s, p)
        t_pre4 = timeit(lambda: ops.preprocess(img, f32=True))
        t_pre3 = timeit(lambda: ops.preprocess_pack3(img, k, s, p))
        print(f"## {k}x{k}/{s} B={B}: preprocess NHWC4 {t_pre4:.0f} us, packed rows {t_pre3:.0f} us")
        print("| tile | NHWC4 us | packed us |")
        print("|---|---:|---:|")
        for tile in [-1] + [t for t in range(100, 110) if t != 101]:
            a = timeit(lambda: ops.conv2d(x4, w4, b, k, k, s, p, True, tile=tile))
            c = timeit(lambda: ops.conv2d_pack3(x3, w3, b, 224, k, k, s, p, True, tile))
            print(f"| {tile} | {a:.0f} | {c:.0f} |", flush=True)
        del x4, x3, img


if __name__ == "__main__":
    main()
