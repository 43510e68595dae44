#!/usr/bin/env python3
"""Time the fused split AlexNet stem (alex_stem.hip) alone at B = 500 under its
ablation variants (set_astem_variant): 0 production, 16 patch loads after the
MFMA loop, 1 no MFMA loop, 2 no epilogue, 4 no patch staging, 6 neither,
64 the phased two-half kernel.  usage: astem_ablate.py [B] [v1,v2,...]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from idunno import ops
    from idunno.models import packed as P

    ext = ops.load()
    dev = torch.device("cuda")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    img = ops.synth_images(1234, 0, B, dev)
    torch.manual_seed(0)
    fs, scale, bias, psum = P.pack_alex_stem_split(torch.randn(64, 3, 11, 11) / 20, torch.randn(64) * 0.1)
    fs, bias, psum = fs.to(dev), bias.to(dev), psum.to(dev)
    variants = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 16, 1, 2, 4, 6, 0]
    outs = {}
    for v in variants:
        ext.set_astem_variant(v)
        for _ in range(3):
            ops.alex_stem_split(img, fs, bias, psum, scale)
        if v in (0, 16, 32, 64):
            outs[v] = ops.alex_stem_split(img, fs, bias, psum, scale)
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ops.alex_stem_split(img, fs, bias, psum, scale)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        print(f"variant {v:2d}: median {statistics.median(ts):7.1f} us  min {min(ts):7.1f} us", flush=True)
    ext.set_astem_variant(64)
    ref = outs.get(0, next(iter(outs.values()), None))
    for v, o in outs.items():
        print(f"variant {v:2d} output identical to variant 0: {torch.equal(o, ref)}", flush=True)


if __name__ == "__main__":
    main()
