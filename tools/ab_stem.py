#!/usr/bin/env python3
"""Same-process A/B of the fused stem's persistent occupancy (workgroups per CU),
at the whole-batch and front-split batch sizes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from idunno import ops
    from idunno.models import build_program

    ext = ops.load()
    s = build_program("resnet18").stem
    w, b = s.w.cuda(), s.b.cuda()
    img = torch.randint(0, 256, (400, 224, 224, 3), dtype=torch.uint8, device="cuda")
    ref = None
    for rnd in range(3):
        for batch in (400, 200):
            for wgs in (2, 4):
                ext.set_stem_workgroups_per_cu(wgs)
                x = img[:batch]
                out = ops.stem_fused(x, w, b)
                if batch == 400:
                    if ref is None:
                        ref = out.clone()
                    assert torch.equal(out, ref), "occupancy changed the result"
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                for _ in range(20):
                    ops.stem_fused(x, w, b)
                en.record()
                torch.cuda.synchronize()
                print(f"round {rnd} batch {batch} wgs/CU {wgs}: {st.elapsed_time(en) / 20 * 1e3:7.1f} us", flush=True)
    ext.set_stem_workgroups_per_cu(4)


if __name__ == "__main__":
    main()
