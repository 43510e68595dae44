#!/usr/bin/env python3
"""Host time of a fresh 60 MB device allocation (+ torch.cat into it) on the
compute stream while HbmStager copies shards on its side stream (thread), vs
with the device idle: does a caching-allocator miss block behind in-flight
H2D copies?"""
import os
import sys
import tempfile
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from idunno.runtime.data import HbmStager

    dev = torch.device("cuda")
    n = 500 * 224 * 224 * 3
    d = tempfile.mkdtemp(prefix="alloc_probe_")
    paths = []
    rng = np.random.default_rng(0)
    for k in range(8):
        p = os.path.join(d, f"s{k}")
        with open(p, "wb") as f:
            f.write(rng.integers(0, 255, n, dtype=np.uint8).tobytes())
        paths.append(p)
    st = HbmStager(dev)
    a = torch.randint(0, 255, (2 * n,), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def cats(tag, k0):
        ts = []
        for i in range(6):
            m = 60_000_000 + (k0 + i) * 4_194_304          # a size no cached block fits
            t0 = time.perf_counter()
            out = torch.cat([a[:m // 2], a[n:n + m - m // 2]])
            ts.append((time.perf_counter() - t0) * 1e3)
            del out
        print(f"{tag}: cat host ms {[round(t, 2) for t in ts]}", flush=True)

    cats("idle", 0)
    keep = []
    th = threading.Thread(target=lambda: keep.extend(st._stage_file(p, (n,))[0] for p in paths))
    th.start()
    time.sleep(0.002)
    cats("during staging", 10)
    th.join()
    torch.cuda.synchronize()
    keep.clear()
    big = torch.empty(int(1.2e9), dtype=torch.uint8, device=dev)
    del big                                                  # a cached 1.2 GB block
    th = threading.Thread(target=lambda: keep.extend(st._stage_file(p, (n,))[0] for p in paths))
    th.start()
    time.sleep(0.002)
    cats("during staging, allocator pre-warmed", 20)
    th.join()
    for p in paths:
        os.unlink(p)
    os.rmdir(d)


if __name__ == "__main__":
    main()
