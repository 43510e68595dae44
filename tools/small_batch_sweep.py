#!/usr/bin/env python3
"""Per-layer kernel choice for the split (fp32-accurate) ResNet18 forward at a
small per-GPU batch -- the strong-scaling chunk of one 400-image query over 8
GPUs is 50 images.  For every distinct conv shape: the
default route, the band kernel (tile 70) where it applies, the im2col tiles
with forced split-K slices, and the layer-1 row kernel (tile 50), as one JSON
line per layer plus a summary of the best choice.

usage: python tools/small_batch_sweep.py [--batch 50] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tools.bench_layers import layer_shapes  # noqa: E402


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models.packed import pack_split_weight, split_eligible

    ops.load()
    dev = "cuda"
    tot_def = tot_best = 0.0
    for name, B, h, c in layer_shapes("resnet18", a.batch):
        if not split_eligible(c.cin, c.cout):
            continue
        w = torch.randn(c.cout, c.cin, c.kh, c.kw) / (c.cin * c.kh * c.kw) ** 0.5
        b = torch.zeros(c.cout, device=dev)
        sw, scale = pack_split_weight(w)
        sw = sw.to(dev)
        xs = ops.split_from_f32(torch.randn(B, h, h, c.cin, device=dev))
        ho = (h + 2 * c.pad - c.kh) // c.stride + 1
        rs = ops.split_from_f32(torch.randn(B, ho, ho, c.cout, device=dev)) if "res" in name else None
        run = lambda **kw: ops.conv2d_split(xs, sw, b, scale, c.kh, c.kw, c.stride, c.pad, True,  # noqa: E731
                                            residual=rs, **kw)
        r = {"layer": name, "H": h, "cin": c.cin, "cout": c.cout, "k": c.kh, "s": c.stride,
             "default": timeit(lambda: run(), a.iters)}
        opts = []
        if c.kh == 3 and c.stride == 1:
            opts.append(("band", dict(tile=70)))
            opts.append(("c64", dict(tile=50)))
        for t in (27, 36, 42, 34, 38):
            for ks in (1, 2, 4, 8):
                if ks > 1 and t not in (27, 36, 42):
                    continue
                opts.append((f"t{t}k{ks}", dict(tile=t, ksplit=ks)))
        for label, kw in opts:
            try:
                r[label] = timeit(lambda: run(**kw), a.iters)
            except RuntimeError:
                pass
        best = min((v, k) for k, v in r.items() if isinstance(v, float))
        r["best"], r["best_us"] = best[1], best[0]
        tot_def += r["default"]
        tot_best += best[0]
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    print(json.dumps({"batch": a.batch, "sum_default_us": round(tot_def, 1), "sum_best_us": round(tot_best, 1)}))


if __name__ == "__main__":
    main()
