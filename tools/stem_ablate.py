#!/usr/bin/env python3
"""Time the fused stem (``--split``: the split-fp16 stem) with parts of its work ablated (profiling only; the
ablated outputs are wrong): where does a tile's time go?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from idunno import ops
    from idunno.models import build_program

    ext = ops.load()
    split = "--split" in sys.argv        # the split-fp16 (fp32-accurate) stem instead of the fp16 one
    if "--reg" in sys.argv:              # --reg N: the register-pooled split stem, N workgroups per CU
        ext.set_stem_split_reg(int(sys.argv[sys.argv.index("--reg") + 1]))
    p = build_program("resnet18", dtype="fp32" if split else "fp16")
    s = p.stem
    img = torch.randint(0, 256, (400, 224, 224, 3), dtype=torch.uint8, device="cuda")
    w, b = s.w.cuda(), s.b.cuda()
    if split:
        fs, fb, fp = s.fs.cuda(), s.fs_bias.cuda(), s.fs_psum.cuda()
        run = lambda: ops.stem_split(img, fs, fb, fp, s.fs_scale)
    else:
        run = lambda: ops.stem_fused(img, w, b)
    names = {0: "full", 1: "no pool", 2: "no MFMA", 4: "no patch normalise", 8: "no conv epilogue",
             16: "no patch loads", 3: "no pool+MFMA", 7: "no pool+MFMA+normalise", 15: "+ no epilogue",
             31: "none (tile loop, barriers)"}
    for rnd in range(2):
        for mode, name in names.items():
            ext.set_stem_ablation(mode)
            run()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(10):
                run()
            en.record()
            torch.cuda.synchronize()
            if rnd:
                print(f"{name:22s} {st.elapsed_time(en) / 10 * 1000:8.1f} us", flush=True)
    ext.set_stem_ablation(0)


if __name__ == "__main__":
    main()
