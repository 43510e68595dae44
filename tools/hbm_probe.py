#!/usr/bin/env python3
"""HBM bandwidth probe: what a plain read+write stream reaches on this GPU
(torch copy_ / add on 1-2 GB tensors), as the ceiling the memory-bound
streaming 1x1 kernels are compared against."""
import torch


def bw(fn, nbytes, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    return nbytes / (ms * 1e-3) / 1e12, ms


def main():
    n = 512 * 1024 * 1024                    # 1 GiB of fp16
    a = torch.randn(n, device="cuda", dtype=torch.float16)
    b = torch.empty_like(a)
    c = torch.randn(n, device="cuda", dtype=torch.float16)
    print("copy  (1R+1W, 2 GiB): %.2f TB/s  %.3f ms" % bw(lambda: b.copy_(a), 2 * a.numel() * 2))
    print("add   (2R+1W, 3 GiB): %.2f TB/s  %.3f ms" % bw(lambda: torch.add(a, c, out=b), 3 * a.numel() * 2))
    print("read  (sum,  1 GiB):  %.2f TB/s  %.3f ms" % bw(lambda: a.sum(dtype=torch.float32), a.numel() * 2))
    print("fill  (1W,   1 GiB):  %.2f TB/s  %.3f ms" % bw(lambda: b.fill_(1.0), a.numel() * 2))


if __name__ == "__main__":
    main()
