#!/usr/bin/env python3
"""Per-layer timing of the split-fp16 (fp32-accurate) conv (conv_glds SPLIT) at
the model's layer shapes: every split tile id vs the default pick, next to the
all-f32-MFMA kernel the fp32 path used before (Winograd v3 for 3x3/s1, direct
conv_f32 otherwise) and the fp16 default, interleaved in one process.
Prints a markdown table (us, and TF/s of useful fp32 FLOPs).

usage: python tools/bench_layers_split.py [--batch 400] [--model resnet18] [--tiles 24,26,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tools.bench_layers import layer_shapes  # noqa: E402
from tools.bench_layers_f32 import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--tiles", default="26,27,34,36,38,42")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models.packed import pack_conv_weight, pack_split_weight, split_eligible, wino_weight

    ops.load()
    dev = "cuda"
    tiles = [int(t) for t in a.tiles.split(",")]
    rows = []
    tot = {"def": 0.0, "best": 0.0, "f32": 0.0}
    if a.model == "alexnet":
        from types import SimpleNamespace as NS
        shapes = [(f"conv{i}", a.batch, h, NS(cin=ci, cout=co, kh=k, kw=k, stride=1, pad=k // 2))
                  for i, h, ci, co, k in ((2, 27, 64, 192, 5), (3, 13, 192, 384, 3), (4, 13, 384, 256, 3),
                                          (5, 13, 256, 256, 3))]
    else:
        shapes = layer_shapes(a.model, a.batch)
    for name, B, h, c in shapes:
        if not split_eligible(c.cin, c.cout):
            continue
        w = torch.randn(c.cout, c.cin, c.kh, c.kw) / (c.cin * c.kh * c.kw) ** 0.5
        b = torch.zeros(c.cout, device=dev)
        sw, scale = pack_split_weight(w)
        sw = sw.to(dev)
        x = torch.randn(B, h, h, c.cin, device=dev)
        xs = ops.split_from_f32(x)
        ho = (h + 2 * c.pad - c.kh) // c.stride + 1
        res = torch.randn(B, ho, ho, c.cout, device=dev) if "res" in name else None
        rs = ops.split_from_f32(res) if res is not None else None
        flops = 2.0 * B * ho * ho * c.cout * c.cin * c.kh * c.kw
        r = {"layer": name, "H": h, "cin": c.cin, "cout": c.cout, "k": c.kh, "s": c.stride,
             "default": ops.pick_tile_split(B * ho * ho, c.cout)}
        for t in tiles:
            try:
                r[t] = timeit(lambda: ops.conv2d_split(xs, sw, b, scale, c.kh, c.kw, c.stride, c.pad, True,
                                                       residual=rs, tile=t))
            except RuntimeError as e:
                print(f"{name} tile {t}: {e}", file=sys.stderr)
        r["def_us"] = timeit(lambda: ops.conv2d_split(xs, sw, b, scale, c.kh, c.kw, c.stride, c.pad, True,
                                                      residual=rs))
        # the all-f32-MFMA kernel of the same layer
        if c.kh == 3 and c.stride == 1 and ops.wino_supported(h, h, c.cin, c.cout):
            u = wino_weight(w).to(dev)
            r["f32_us"] = timeit(lambda: ops.conv2d_wino(x, u, b, True, res, 3))
        else:
            pw, _ = pack_conv_weight(w, "fp32")
            pw = pw.to(dev)
            r["f32_us"] = timeit(lambda: ops.conv2d(x, pw, b, c.kh, c.kw, c.stride, c.pad, True, residual=res))
        # fp16 default (fp16 activations, reference for the byte/MFMA ratio)
        ph, _ = pack_conv_weight(w, "fp16")
        ph, xh = ph.to(dev), x.half()
        rh = res.half() if res is not None else None
        r["f16_us"] = timeit(lambda: ops.conv2d(xh, ph, b, c.kh, c.kw, c.stride, c.pad, True, residual=rh))
        timed = [(v, k) for k, v in r.items() if isinstance(k, int)]
        best_us, best_t = min(timed) if timed else (r["def_us"], r["default"])   # no listed tile fits the shape
        r["best_tile"], r["best_us"] = best_t, best_us
        r["tf_best"] = flops / best_us / 1e6
        tot["def"] += r["def_us"]
        tot["best"] += best_us
        tot["f32"] += r["f32_us"]
        rows.append(r)
        print(json.dumps(r), flush=True)
    print("\n| layer | H | cin | cout | k/s | default | def us | best tile | best us | best TF/s | f32-MFMA us |"
          " split/f32 | fp16 us | split/fp16 |")
    print("|---|---:|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for r in rows:
        print(f"| {r['layer']} | {r['H']} | {r['cin']} | {r['cout']} | {r['k']}/{r['s']} | {r['default']} | "
              f"{r['def_us']:.0f} | {r['best_tile']} | {r['best_us']:.0f} | {r['tf_best']:.0f} | {r['f32_us']:.0f} |"
              f" {r['best_us'] / r['f32_us']:.2f} | {r['f16_us']:.0f} | {r['best_us'] / r['f16_us']:.2f} |")
    print(f"\nunique layers: split default {tot['def']:.0f} us, split best {tot['best']:.0f} us, "
          f"f32-MFMA {tot['f32']:.0f} us")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
