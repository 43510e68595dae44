#!/usr/bin/env python3
"""fp16 AlexNet conv1 (11x11/4, B=500): NHWC4 + conv_igemm vs packed rows +
conv_glds pack3 per tile, and the two preprocess kernels."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wino_variants import timeit  # noqa: E402


def main():
    from idunno import ops
    from idunno.models.packed import pack_conv_weight, pack_conv_weight_p3

    ops.load()
    B, k, s, p = 500, 11, 4, 2
    img = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
    w = torch.randn(64, 3, k, k) / (3 * k * k) ** 0.5
    b = torch.zeros(64, device="cuda")
    w4 = pack_conv_weight(w, "fp16")[0].cuda()
    w3 = pack_conv_weight_p3(w, "fp16").cuda()
    x4 = ops.preprocess(img)
    x3 = ops.preprocess_pack3(img, k, s, p, f16=True)
    print(f"preprocess NHWC4 {timeit(lambda: ops.preprocess(img)):.0f} us, "
          f"packed rows {timeit(lambda: ops.preprocess_pack3(img, k, s, p, f16=True)):.0f} us")
    print(f"NHWC4 conv (default) {timeit(lambda: ops.conv2d(x4, w4, b, k, k, s, p, True)):.0f} us")
    for t in (-1, 23, 27, 31, 33, 35):
        print(f"packed tile {t}: {timeit(lambda: ops.conv2d_pack3(x3, w3, b, 224, k, k, s, p, True, t)):.0f} us",
              flush=True)


if __name__ == "__main__":
    main()
