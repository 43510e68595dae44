#!/usr/bin/env python3
"""Does host -> HBM staging (HbmStager, side stream) run under the forwards?
Times N ResNet18 graph replays alone, 8 shard stagings alone, and both
together (staging on a thread), with the shard buffers allocated during the
staging (as SdfsSource does) or beforehand (--prealloc arm).

usage: python tools/overlap_probe.py [--iters 12]
"""
import argparse
import os
import sys
import tempfile
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--shards", type=int, default=8)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program
    from idunno.runtime.data import HbmStager

    dev = torch.device("cuda")
    r = HipRunner(build_program("resnet18", dtype="fp32"), dev)
    shard = ops.synth_images(1234, 0, 400, dev)
    _s, run = r.capture_window(shard, 400)
    n = 500 * 224 * 224 * 3
    d = tempfile.mkdtemp(prefix="ovl_probe_")
    paths = []
    rng = np.random.default_rng(0)
    for k in range(a.shards):
        p = os.path.join(d, f"s{k}")
        with open(p, "wb") as f:
            f.write(rng.integers(0, 255, n, dtype=np.uint8).tobytes())
        paths.append(p)
    st = HbmStager(dev)

    def fwd():
        for _ in range(a.iters):
            run()
        torch.cuda.synchronize()

    def stage(pre):
        outs = []
        for i, p in enumerate(paths):
            if pre is not None:
                t, ev = pre[i], None
                with open(p, "rb") as f:
                    pass
                t2, ev = st._stage_file(p, (n,))
                outs.append(t2)
            else:
                outs.append(st._stage_file(p, (n,))[0])
        torch.cuda.synchronize()
        return outs

    for _ in range(3):
        fwd()
    stage(None)
    res = {}
    for rep in range(3):
        for arm in ("fwd", "stage", "both", "both_cached_alloc"):
            torch.cuda.synchronize()
            if arm == "both_cached_alloc":
                # make the allocator hold enough free blocks first: stage, free, restage
                keep = stage(None)
                del keep
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            if arm == "fwd":
                fwd()
            elif arm == "stage":
                keep = stage(None)
                del keep
            else:
                th = threading.Thread(target=lambda: stage(None))
                th.start()
                fwd()
                th.join()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) * 1e3
            res.setdefault(arm, []).append(dt)
            print(f"{arm}: {dt:.1f} ms", flush=True)
    for k, v in res.items():
        print(f"{k}: min {min(v):.1f} ms", flush=True)
    for p in paths:
        os.unlink(p)
    os.rmdir(d)


if __name__ == "__main__":
    main()
