#!/usr/bin/env python3
"""Host-time probe of one collective-round chunk launch on the GPU
(``HipExecutor.run_packed`` as ``RoundPlane._run_chunk`` calls it): 2 rounds
in flight, per-step host microseconds of every call on the launch path.

usage: python tools/system_launch_probe.py [--rounds 40] [--batch 400]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--direct", action="store_true", help="hipGraphLaunch via ops.graph_launch, not CUDAGraph.replay")
    a = ap.parse_args()
    from idunno import ops
    from idunno.runtime.data import SyntheticSource
    from idunno.runtime.executor import HipExecutor

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ex = HipExecutor(dev, seed=0)
    src = SyntheticSource(1, dev)
    sends = [torch.zeros(a.batch + 2, 2, dtype=torch.int32, device=dev) for _ in range(2)]
    r = ex.runner(a.model)
    for sl in range(2):                      # capture both graphs first
        r.capture(a.batch, packed=sends[sl][: a.batch])
    torch.cuda.synchronize()
    T = {k: [] for k in ("stage", "enter", "ev0", "lookup", "copy", "replay", "tail", "total", "wait")}
    done = []
    for q in range(a.rounds):
        if len(done) >= 2:
            t = time.perf_counter()
            done.pop(0).synchronize()
            T["wait"].append(time.perf_counter() - t)
        t0 = time.perf_counter()
        imgs = src.get(q * a.batch, (q + 1) * a.batch - 1)
        t1 = time.perf_counter()
        packed = sends[q % 2][: a.batch]
        with torch.cuda.device(dev), ex.run_lock:
            s = ex._enter(imgs)
            t2 = time.perf_counter()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                ev0.record(s)
                t3 = time.perf_counter()
                sin, replay = r.capture(a.batch, packed=packed)
                t4 = time.perf_counter()
                sin.copy_(imgs)
                t5 = time.perf_counter()
                if a.direct:
                    g = r._graphs[r._capture_key(a.batch, packed, 0)][0]
                    ops.load().graph_launch(g.raw_cuda_graph_exec())
                else:
                    replay()
                t6 = time.perf_counter()
                ev1.record(s)
            torch.cuda.current_stream(dev).wait_stream(s)
            t7 = time.perf_counter()
        ev = torch.cuda.Event()
        ev.record()
        done.append(ev)
        for k, x, y in (("stage", t0, t1), ("enter", t1, t2), ("ev0", t2, t3), ("lookup", t3, t4), ("copy", t4, t5),
                        ("replay", t5, t6), ("tail", t6, t7), ("total", t0, t7)):
            T[k].append(y - x)
    torch.cuda.synchronize()
    for k, v in T.items():
        v = v[4:]
        if v:
            print(f"{k:8s} median {1e6 * statistics.median(v):9.1f} us   max {1e6 * max(v):9.1f} us")


if __name__ == "__main__":
    main()
