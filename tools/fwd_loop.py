#!/usr/bin/env python3
"""Time (and give rocprofv3 something to trace) the captured forward of one
model: ``iters`` hipGraph replays of the whole forward over a resident shard.

usage: python tools/fwd_loop.py [--model resnet18] [--batch 400] [--dtype fp32] [--iters 25]
                                [--attr name=value ...]   (HipRunner attributes, ints or true/false)
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--iters", type=int, default=25)
    ap.add_argument("--attr", action="append", default=[])
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program

    dev = torch.device("cuda")
    r = HipRunner(build_program(a.model, dtype=a.dtype), dev)
    for kv in a.attr:
        k, v = kv.split("=")
        setattr(r, k, {"true": True, "false": False, "none": None}.get(v.lower(), int(v) if v.lstrip("-").isdigit() else v))
    shard = ops.synth_images(1234, 0, a.batch, dev)
    _s, run = r.capture_window(shard, a.batch)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    print(f"{a.model} b{a.batch} {a.dtype} {a.attr}: {dt * 1e3:.3f} ms/forward, {a.batch / dt:.0f} img/s", flush=True)


if __name__ == "__main__":
    main()
