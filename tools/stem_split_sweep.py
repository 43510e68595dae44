#!/usr/bin/env python3
"""Split-fp16 packed-row stem (conv_glds P3+SPLIT): time every tile at the
ResNet stem (7x7/2) and AlexNet conv1 (11x11/4) shapes, plus the split
preprocess and the f32 stem it replaces.  usage: python tools/stem_split_sweep.py [--batch 400]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_layers_f32 import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=400)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models.packed import pack_conv_weight_p3, pack_split_weight_p3

    ops.load()
    dev = "cuda"
    img = ops.synth_images(0, 0, a.batch, dev)
    print("| stem | tile | conv us | preprocess us |")
    print("|---|---:|---:|---:|")
    for name, kh, s, p in (("resnet 7x7/2", 7, 2, 3), ("alexnet 11x11/4", 11, 4, 2)):
        w = torch.randn(64, 3, kh, kh) / (3 * kh * kh) ** 0.5
        b = torch.zeros(64, device=dev)
        sp3, sc = pack_split_weight_p3(w)
        sp3 = sp3.to(dev)
        x3 = ops.preprocess_pack3_split(img, kh, s, p)
        pre = timeit(lambda: ops.preprocess_pack3_split(img, kh, s, p))
        for t in (23, 27, 33, 35, 37):
            us = timeit(lambda: ops.conv2d_pack3_split(x3, sp3, b, sc, 224, kh, kh, s, p, True, tile=t))
            print(f"| {name} split | {t} | {us:.0f} | {pre:.0f} |", flush=True)
        if kh == 7:
            from idunno.models.packed import pack_stem_split
            fs, fsc, fsb, fsp = (t.to(dev) if torch.is_tensor(t) else t for t in pack_stem_split(w))
            for niw in (2, 1):
                ops.load().set_stem_split_niw(niw)
                us = timeit(lambda: ops.stem_split(img, fs, fsb, fsp, fsc))
                print(f"| {name} fused split stem (+relu+maxpool, no preprocess), {niw} cout fragments/wave | - |"
                      f" {us:.0f} | 0 |", flush=True)
            ops.load().set_stem_split_niw(1)
            x = torch.empty(a.batch, 112, 112, 64, device=dev)
            us = timeit(lambda: ops.maxpool2d_split(x, 3, 2, 1))
            print(f"| maxpool f32 -> split (unfused path) | - | {us:.0f} | - |", flush=True)
        p3 = pack_conv_weight_p3(w, "fp32").to(dev)
        x3f = ops.preprocess_pack3(img, kh, s, p)
        pref = timeit(lambda: ops.preprocess_pack3(img, kh, s, p))
        us = timeit(lambda: ops.conv2d_pack3(x3f, p3, b, 224, kh, kh, s, p, True))
        print(f"| {name} f32 | default | {us:.0f} | {pref:.0f} |", flush=True)


if __name__ == "__main__":
    main()
