#!/usr/bin/env python3
"""Per-layer timing of the fp32 conv kernel (conv_f32.hip) at the model's
layer shapes: every tile id vs the default pick vs PyTorch fp32 (MIOpen,
channels_last), interleaved in one process.  Prints a markdown table with
us and TF/s (useful FLOPs) per layer and tile.

usage: python tools/bench_layers_f32.py [--batch 400] [--model resnet18] [--tiles 100,101,...]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tools.bench_layers import layer_shapes  # noqa: E402


def timeit(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) * 1000 / iters   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--tiles", default="100,101,102,103,104,105,106,107,108,109")
    ap.add_argument("--json", default=None)
    ap.add_argument("--torch", action="store_true", help="also time PyTorch fp32 conv")
    a = ap.parse_args()
    from idunno import ops
    ops.load()
    dev = "cuda"
    tiles = [int(t) for t in a.tiles.split(",")]
    from idunno.models.packed import Conv, pack_conv_weight

    rows = []
    tot_best = tot_def = 0.0
    for name, B, h, c16 in layer_shapes(a.model, a.batch):
        w = torch.randn(c16.cout, c16.cin, c16.kh, c16.kw) / (c16.cin * c16.kh * c16.kw) ** 0.5
        pw, small = pack_conv_weight(w, "fp32")
        c = Conv(pw.to(dev), torch.zeros(c16.cout, device=dev), c16.cin, c16.cout, c16.kh, c16.kw,
                 c16.stride, c16.pad, True, small)
        cin = 4 if c.small else c.cin
        x = torch.randn(B, h, h, cin, device=dev)
        ho = (h + 2 * c.pad - c.kh) // c.stride + 1
        res = torch.randn(B, ho, ho, c.cout, device=dev) if "res" in name else None
        flops = 2.0 * B * ho * ho * c.cout * c.cin * c.kh * c.kw
        r = {"layer": name, "H": h, "cin": c.cin, "cout": c.cout, "k": c.kh, "s": c.stride,
             "default": ops.pick_tile_f32(B * ho * ho, c.cout, c.w.shape[1], c.small)}
        for t in tiles:
            if c.small and t == 101:
                continue
            try:
                us = timeit(lambda: ops.conv2d(x, c.w, c.b, c.kh, c.kw, c.stride, c.pad, True, residual=res, tile=t))
            except RuntimeError as e:
                print(f"{name} tile {t}: {e}", file=sys.stderr)
                continue
            r[t] = us
        if c.kh == 3 and c.stride == 1 and ops.wino_supported(h, h, c.cin, c.cout):
            from idunno.models.packed import wino_weight

            u = wino_weight(w).to(dev)
            for var in (0, 1, 2):
                r[f"wino{var}_us"] = timeit(lambda: ops.conv2d_wino(x, u, c.b, True, res, var))
            r["wino_tf"] = flops / min(r["wino0_us"], r["wino1_us"], r["wino2_us"]) / 1e6
        us_def = timeit(lambda: ops.conv2d(x, c.w, c.b, c.kh, c.kw, c.stride, c.pad, True, residual=res))
        r["def_us"] = us_def
        if a.torch and not c.small:
            xt = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            wt = torch.randn(c.cout, c.cin, c.kh, c.kw, device=dev).contiguous(memory_format=torch.channels_last)
            r["torch_us"] = timeit(lambda: F.conv2d(xt, wt, None, c.stride, c.pad))
        best = min(v for k, v in r.items() if isinstance(k, int))
        r["best_tile"] = min((v, k) for k, v in r.items() if isinstance(k, int))[1]
        r["tf_best"] = flops / best / 1e6
        r["tf_def"] = flops / us_def / 1e6
        tot_best += best
        tot_def += us_def
        rows.append(r)
        print(json.dumps(r), flush=True)
    print(f"\n| layer | H | cin | cout | k/s | default | def us | def TF/s | best tile | best us | best TF/s |"
          " wino4 us | wino8 us | wino4p us | wino eff. TF/s |" + (" torch us |" if a.torch else ""))
    print("|---|---:|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|" + ("---:|" if a.torch else ""))
    for r in rows:
        best = min(v for k, v in r.items() if isinstance(k, int))
        print(f"| {r['layer']} | {r['H']} | {r['cin']} | {r['cout']} | {r['k']}/{r['s']} | {r['default']} | "
              f"{r['def_us']:.0f} | {r['tf_def']:.1f} | {r['best_tile']} | {best:.0f} | {r['tf_best']:.1f} |"
              f" {r.get('wino0_us', float('nan')):.0f} | {r.get('wino1_us', float('nan')):.0f} |"
              f" {r.get('wino2_us', float('nan')):.0f} |"
              f" {r.get('wino_tf', float('nan')):.1f} |"
              + (f" {r.get('torch_us', float('nan')):.0f} |" if a.torch else ""))
    print(f"\nunique layers: default sum {tot_def:.0f} us, best-tile sum {tot_best:.0f} us")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
