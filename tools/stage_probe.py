#!/usr/bin/env python3
"""Host -> HBM staging rates of SDFS-shard-sized files on this box (page-cache
resident, as after an SDFS put): the pinned ping-pong preadv path
(HbmStager._stage_file) at several reader-thread counts, against mapping the
file and registering the mapping with the HIP runtime (hipHostRegister: the DMA
engine reads the page-cache pages, no host copy).

usage: python tools/stage_probe.py [--shards 8] [--mb 75]
"""
import argparse
import ctypes
import mmap
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--mb", type=int, default=75)
    a = ap.parse_args()
    from idunno.runtime.data import HbmStager

    dev = torch.device("cuda")
    torch.empty(1, device=dev)
    d = tempfile.mkdtemp(prefix="stage_probe_")
    n = a.mb << 20
    paths = []
    rng = np.random.default_rng(0)
    for k in range(a.shards):
        p = os.path.join(d, f"s{k}")
        with open(p, "wb") as f:
            f.write(rng.integers(0, 255, n, dtype=np.uint8).tobytes())
        paths.append(p)
    tot = n * a.shards
    print(f"{a.shards} files x {a.mb} MB in {d}", flush=True)
    try:
        for th in (4, 8, 16):
            st = HbmStager(dev)
            st.READ_THREADS = th
            for rep in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                outs = [st._stage_file(p, (n,))[0] for p in paths]
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print(f"pinned preadv, {th} threads, pass {rep}: {tot / dt / 1e9:.2f} GB/s ({dt * 1e3:.1f} ms)", flush=True)
            del outs
        # mmap + hipHostRegister + one DMA per file
        rt = torch._C._cudart
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            treg = tcp = 0.0
            keep = []
            for p in paths:
                fd = os.open(p, os.O_RDWR)
                mm = mmap.mmap(fd, n, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
                os.close(fd)
                addr = ctypes.addressof(ctypes.c_char.from_buffer(mm))
                t1 = time.perf_counter()
                err = rt.cudaHostRegister(addr, n, 0)
                treg += time.perf_counter() - t1
                if int(err) != 0:
                    print(f"hostRegister failed: {err}", flush=True)
                    return
                src = torch.frombuffer(mm, dtype=torch.uint8)
                out = torch.empty(n, dtype=torch.uint8, device=dev)
                t1 = time.perf_counter()
                out.copy_(src, non_blocking=True)
                tcp += time.perf_counter() - t1
                keep.append((mm, addr, src, out))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ok = all(torch.equal(o[:4096].cpu(), s[:4096]) for _m, _a, s, o in keep[:2])
            for mm, addr, src, out in keep:
                rt.cudaHostUnregister(addr)
                del src
                mm.close()
            print(f"mmap + hostRegister, pass {rep}: {tot / dt / 1e9:.2f} GB/s ({dt * 1e3:.1f} ms; register "
                  f"{treg * 1e3:.1f} ms, copy issue {tcp * 1e3:.1f} ms; data ok {ok})", flush=True)
    finally:
        for p in paths:
            os.unlink(p)
        os.rmdir(d)


if __name__ == "__main__":
    main()
