#!/usr/bin/env python3
"""Vendor-library baseline on the same GPU: the reference model definitions run
through PyTorch-ROCm (MIOpen convs, hipBLASLt FC), fp16 channels_last, batch B,
preprocess + forward + softmax-top1, optionally hipGraph-captured.  This is the
"what would a straight PyTorch port get" number our HIP path must beat.

usage: python tools/bench_torch_baseline.py [--model resnet18] [--batch 400] [--iters 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-graph", action="store_true")
    a = ap.parse_args()
    from idunno.models import reference as ref

    torch.backends.cudnn.benchmark = True
    m = ref.build(a.model, seed=0).cuda().half().to(memory_format=torch.channels_last)
    img = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device="cuda")

    def step():
        with torch.no_grad():
            x = ref.preprocess_u8(img).half().contiguous(memory_format=torch.channels_last)
            p = torch.softmax(m(x).float(), 1)
            return p.max(1)

    ref.preprocess_u8(img[:1])   # materialise the cached normalisation constants
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    fn = step
    if not a.no_graph:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            step()
        fn = g.replay
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    out = {"what": "pytorch-rocm (MIOpen) baseline", "model": a.model, "batch": a.batch,
           "ms_per_batch": round(dt * 1e3, 3), "images_per_s": round(a.batch / dt, 1), "graph": not a.no_graph}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
