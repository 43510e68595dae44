#!/usr/bin/env python3
"""Run the fused stem a few times at B=400 (a short program for rocprofv3 --pmc)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from idunno import ops
    from idunno.models import build_program

    s = build_program("resnet18").stem
    w, b = s.w.cuda(), s.b.cuda()
    img = torch.randint(0, 256, (400, 224, 224, 3), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        ops.stem_fused(img, w, b)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
