#!/usr/bin/env python3
"""Library ceilings for the split-fp32 conv layers (ResNet18, B = 400).

For every 3x3 / 1x1 conv shape of the split path this times, on one MI355X:
  * hipBLASLt fp16 GEMM (torch.mm) of the equivalent work: M = B*Ho*Wo pixels,
    N = Cout, K = 3 * KH*KW*Cin (a split product is 3 f16 MACs), operands
    already materialised (no im2col cost charged to the library);
  * MIOpen conv2d in fp16 (channels_last) and fp32 of the same layer;
  * our split conv (ops.conv2d_split via the packed program's tile pick),
and prints a markdown table in TFLOP/s of f16-equivalent MFMA work.
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3     # us


SHAPES = [  # (name, H(in), Cin, Cout, k, stride)
    ("l1 3x3", 56, 64, 64, 3, 1),
    ("l2 3x3/2", 56, 64, 128, 3, 2),
    ("l2 3x3", 28, 128, 128, 3, 1),
    ("l3 3x3/2", 28, 128, 256, 3, 2),
    ("l3 3x3", 14, 256, 256, 3, 1),
    ("l4 3x3/2", 14, 256, 512, 3, 2),
    ("l4 3x3", 7, 512, 512, 3, 1),
    ("l2 ds 1x1/2", 56, 64, 128, 1, 2),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models.packed import pack_split_weight

    ops.load()
    dev = "cuda"
    B = a.batch
    print(f"### Library ceilings vs split conv, B = {B} (us per launch; TF/s of f16-equivalent MFMA work = 3 x fp32 MACs x 2)\n")
    print("| layer | M | N | K (3x) | hipBLASLt fp16 GEMM | MIOpen fp16 conv | MIOpen fp32 conv | split conv (ours) |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    torch.manual_seed(0)
    for name, H, Cin, Cout, k, s in SHAPES:
        pad = k // 2
        Ho = (H + 2 * pad - k) // s + 1
        M, N, K = B * Ho * Ho, Cout, 3 * k * k * Cin
        flop = 2.0 * M * N * K
        A = torch.randn(M, K, device=dev, dtype=torch.float16)
        Bm = torch.randn(K, N, device=dev, dtype=torch.float16)
        t_mm = timeit(lambda: torch.mm(A, Bm), a.iters)
        del A, Bm
        x16 = torch.randn(B, Cin, H, H, device=dev, dtype=torch.float16).to(memory_format=torch.channels_last)
        w16 = torch.randn(Cout, Cin, k, k, device=dev, dtype=torch.float16).to(memory_format=torch.channels_last)
        t_c16 = timeit(lambda: torch.nn.functional.conv2d(x16, w16, stride=s, padding=pad), a.iters)
        x32, w32 = x16.float(), w16.float()
        t_c32 = timeit(lambda: torch.nn.functional.conv2d(x32, w32, stride=s, padding=pad), max(3, a.iters // 4))
        del x16, w16
        # ours: split layout [B][H][W][2*Cin] halfs, weights via the split packer
        xs = ops.split_from_f32(x32.permute(0, 2, 3, 1).contiguous())
        sw, scale = pack_split_weight((w32 / (Cin * k * k) ** 0.5).cpu())
        sw, bias = sw.to(dev), torch.zeros(Cout, device=dev)
        t_ours = timeit(lambda: ops.conv2d_split(xs, sw, bias, scale, k, k, s, pad, True), a.iters)
        del x32, w32, xs
        tf = lambda t: flop / (t * 1e-6) / 1e12  # noqa: E731
        print(f"| {name} | {M} | {N} | {K} | {t_mm:.0f} us ({tf(t_mm):.0f} TF) | {t_c16:.0f} us ({tf(t_c16) / 3:.0f} TF fp16) | "
              f"{t_c32:.0f} us | {t_ours:.0f} us ({tf(t_ours):.0f} TF) |", flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
