#!/usr/bin/env python3
"""Same-process A/B of the dual (fused downsample) split conv against the two
separate convs, per ResNet18 stride-2 block shape at B = 400, plus the next
conv reading the dual output's halves in place vs contiguous copies."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1000 / iters)
    return statistics.median(out)


def main():
    from idunno import ops
    from idunno.models import packed as P

    dev = "cuda"
    B = 400
    for H, C, Cout in ((56, 64, 128), (28, 128, 256), (14, 256, 512)):
        torch.manual_seed(0)
        x = ops.split_from_f32(torch.randn(B, H, H, C, device=dev))
        s3, sc3 = P.pack_split_weight(torch.randn(Cout, C, 3, 3) * 0.05)
        s1, sc1 = P.pack_split_weight(torch.randn(Cout, C, 1, 1) * 0.05)
        s2, sc2 = P.pack_split_weight(torch.randn(Cout, Cout, 3, 3) * 0.05)
        s3, s1, s2 = s3.to(dev), s1.to(dev), s2.to(dev)
        b = torch.zeros(Cout, device=dev)
        c2 = s3.shape[1] // 9
        wd = torch.zeros(2 * Cout, s3.shape[1], dtype=s3.dtype, device=dev)
        wd[:Cout] = s3
        wd[Cout:, 4 * c2:5 * c2] = s1
        bd = torch.zeros(2 * Cout, device=dev)
        t_main = timeit(lambda: ops.conv2d_split(x, s3, b, sc3, 3, 3, 2, 1, True))
        t_ds = timeit(lambda: ops.conv2d_split(x, s1, b, sc1, 1, 1, 2, 0, False))
        t_dual = timeit(lambda: ops.conv2d_split_dual(x, wd, bd, sc3, sc1, Cout, 3, 3, 2, 1, True))
        t_dual_full = timeit(lambda: ops.conv2d_split_dual(x, wd, bd, sc3, sc1, Cout, 3, 3, 2, 1, True,
                                                           center_only=False))
        both = ops.conv2d_split_dual(x, wd, bd, sc3, sc1, Cout, 3, 3, 2, 1, True)
        y, r = both[..., :2 * Cout], both[..., 2 * Cout:]
        yc, rc = y.contiguous(), r.contiguous()
        t_next_strided = timeit(lambda: ops.conv2d_split(y, s2, b, sc2, 3, 3, 1, 1, True, residual=r))
        t_next_contig = timeit(lambda: ops.conv2d_split(yc, s2, b, sc2, 3, 3, 1, 1, True, residual=rc))
        print(f"H{H} C{C}->{Cout}: main {t_main:.1f} + ds {t_ds:.1f} = {t_main + t_ds:.1f} us | dual {t_dual:.1f} "
              f"(full-K ds {t_dual_full:.1f}) | next conv strided {t_next_strided:.1f} vs contiguous "
              f"{t_next_contig:.1f} us", flush=True)


if __name__ == "__main__":
    main()
