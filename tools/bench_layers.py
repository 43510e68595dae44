#!/usr/bin/env python3
"""Per-layer conv timing on the GPU: every tile config of the HIP kernels vs
PyTorch's own conv (MIOpen, channels_last fp16) at the ResNet18 / ResNet50
layer shapes, batch B.  Interleaved rounds in one process (§5.4 rule 24).

usage: python tools/bench_layers.py [--batch 400] [--model resnet18] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def layer_shapes(model, B):
    from idunno.models import build_program

    p = build_program(model)
    shapes = []
    h = 224
    def out(h, c):
        return (h + 2 * c.pad - c.kh) // c.stride + 1
    s = p.stem
    shapes.append(("stem", B, h, s))
    h = out(h, s)
    h = (h + 2 - 3) // 2 + 1
    for bi, blk in enumerate(p.blocks):
        hin = h
        for ci, c in enumerate(blk.convs):
            shapes.append((f"b{bi}c{ci}{'+res' if ci == len(blk.convs) - 1 else ''}", B, h, c))
            h = out(h, c)
        if blk.down is not None:
            shapes.append((f"b{bi}ds", B, hin, blk.down))
    uniq, seen = [], set()
    for name, b, hh, c in shapes:
        key = (hh, c.cin, c.cout, c.kh, c.stride, "res" in name)
        if key in seen:
            continue
        seen.add(key)
        uniq.append((name, b, hh, c))
    return uniq


def timeit(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tiles", default="auto,0,1,2,3,10,11,12,13,14,15,16,17,18,19,20,21,22,23")
    ap.add_argument("--json", default=None)
    ap.add_argument("--layers", default=None, help="comma list of layer names to run (default all)")
    ap.add_argument("--no-stem", action="store_true")
    a = ap.parse_args()
    only = set(a.layers.split(",")) if a.layers else None
    from idunno import ops

    ops.load()
    dev = "cuda"
    rows = []
    tiles = [t for t in a.tiles.split(",")]
    # stem: unfused (preprocess + conv + maxpool) vs fused kernel vs torch
    from idunno.models import build_program
    from idunno.models.reference import preprocess_u8
    p = build_program(a.model)
    s = p.stem
    if a.model.startswith("resnet") and not a.no_stem:
        img = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device=dev)
        w, b = s.w.to(dev), s.b.to(dev)
        t_unf = min(timeit(lambda: ops.maxpool2d(ops.conv2d(ops.preprocess(img), w, b, 7, 7, 2, 3, True), 3, 2, 1))
                    for _ in range(a.rounds))
        t_fus = min(timeit(lambda: ops.stem_fused(img, w, b)) for _ in range(a.rounds))
        from idunno.models.packed import unpack_conv_weight
        wr = unpack_conv_weight(s).half().to(dev)
        t_tor = min(timeit(lambda: F.max_pool2d(F.relu(F.conv2d(preprocess_u8(img).half(), wr, b.half(), 2, 3)), 3, 2, 1))
                    for _ in range(a.rounds))
        print(f"stem+pool  unfused {t_unf:8.1f}us  fused {t_fus:8.1f}us  torch {t_tor:8.1f}us", flush=True)
        rows.append({"layer": "stem+maxpool", "us": {"unfused": t_unf, "fused": t_fus, "torch": t_tor}})
    for name, B, h, c in layer_shapes(a.model, a.batch):
        if only is not None and name not in only:
            continue
        cin = 4 if c.small else c.cin
        x = torch.randn(B, h, h, cin, device=dev).half()
        if c.small:
            x[..., 3] = 0
        w, b = c.w.to(dev), c.b.to(dev)
        ho = (h + 2 * c.pad - c.kh) // c.stride + 1
        res = torch.randn(B, ho, ho, c.cout, device=dev).half() if "res" in name else None
        flops = 2.0 * B * ho * ho * c.cout * c.cin * c.kh * c.kw
        res_t = {}
        for _ in range(a.rounds):
            for t in tiles:
                if c.small and t not in ("auto", "0", "1", "2", "3"):
                    continue
                tid = -1 if t == "auto" else int(t)
                if tid in (14, 17) and c.cout % 128:
                    continue
                try:
                    us = timeit(lambda: ops.conv2d(x, w, b, c.kh, c.kw, c.stride, c.pad, True, residual=res, tile=tid))
                except Exception as e:  # noqa: BLE001
                    us = float("nan")
                res_t.setdefault(t, []).append(us)
            # PyTorch / MIOpen reference at the same shape (NHWC fp16)
            xr = x[..., :c.cin].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last) if not c.small \
                else x[..., :3].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            from idunno.models.packed import unpack_conv_weight
            wr = unpack_conv_weight(c).half().to(dev).contiguous(memory_format=torch.channels_last)
            rr = res.permute(0, 3, 1, 2) if res is not None else None
            def tfn():
                y = F.conv2d(xr, wr, b.half(), c.stride, c.pad)
                if rr is not None:
                    y = y + rr
                return F.relu(y)
            res_t.setdefault("torch", []).append(timeit(tfn))
        best = {k: min(v) for k, v in res_t.items()}
        row = {"layer": name, "B": B, "H": h, "cin": c.cin, "cout": c.cout, "k": c.kh, "s": c.stride,
               "gflop": flops / 1e9, "us": best,
               "tflops": {k: (flops / (v * 1e-6) / 1e12 if v == v else None) for k, v in best.items()}}
        rows.append(row)
        ours = {k: v for k, v in best.items() if k != "torch" and v == v}
        kbest = min(ours, key=ours.get)
        print(f"{name:10s} H={h:3d} {c.cin:4d}->{c.cout:4d} k{c.kh}s{c.stride} {flops/1e9:7.1f} GF | "
              f"auto {best.get('auto', float('nan')):8.1f}us best[{kbest}] {ours[kbest]:8.1f}us "
              f"({flops/ours[kbest]/1e6:6.0f} TF/s) | torch {best['torch']:8.1f}us", flush=True)
        print("    " + " ".join(f"{k}:{v:.0f}" for k, v in sorted(best.items(), key=lambda kv: kv[1])), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
