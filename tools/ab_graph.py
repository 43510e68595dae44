#!/usr/bin/env python3
"""Same-process A/B of the whole forward hipGraph: the in-tree extension vs an
alternate build of it (``--alt-so``, e.g. the previous commit's ``_C.so``),
interleaved rounds on one device (cdna_hip_programming §5.4 rule 24; boxes of
the pool differ by several % in wall time, so cross-call numbers do not rank
builds).

usage: python tools/ab_graph.py --alt-so ab/_C_base.so [--model resnet18] [--batch 400] [--dtype fp32]
"""
import argparse
import importlib.util
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def load_alt(path):
    spec = importlib.util.spec_from_file_location("idunno_alt._C", path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alt-so", required=True)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--dtype", default="fp32", help="fp32 (split fp16, the headline) or fp16")
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program
    from idunno.ops import _ext

    dev = torch.device("cuda")
    main_mod = ops.load()
    alt_mod = load_alt(a.alt_so)
    prog = build_program(a.model, dtype=a.dtype)
    shard = ops.synth_images(1234, 0, a.batch, dev)
    runs, outs, keep = {}, {}, []
    for name, mod in (("main", main_mod), ("alt", alt_mod)):
        _ext._mod = mod                        # kernels captured into this graph come from `mod`
        r = HipRunner(prog, dev)
        keep.append(r)                         # the graph holds raw pointers to r's weights
        _start, run = r.capture_window(shard, a.batch)
        runs[name] = run
        cls, prob = run()
        torch.cuda.synchronize()
        outs[name] = (cls.clone(), prob.clone())
    _ext._mod = main_mod
    agree = (outs["main"][0] == outs["alt"][0]).float().mean().item()
    dprob = (outs["main"][1] - outs["alt"][1]).abs().max().item()
    print(f"top-1 agreement main vs alt: {agree:.4f}, max |dprob| {dprob:.2e}", flush=True)
    res = {k: [] for k in runs}
    for _ in range(a.rounds):
        for name, run in runs.items():
            run()
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.iters):
                run()
            t1.record()
            torch.cuda.synchronize()
            res[name].append(t0.elapsed_time(t1) / a.iters)
    for name, v in res.items():
        print(f"{name:5s} {a.model} b{a.batch}: median {statistics.median(v):.4f} ms  min {min(v):.4f} ms  "
              f"({a.batch / statistics.median(v) * 1e3:,.0f} img/s)  rounds {[round(x, 4) for x in v]}", flush=True)
    m, b = statistics.median(res["main"]), statistics.median(res["alt"])
    print(f"main vs alt: {100 * (b / m - 1):+.2f}% throughput", flush=True)


if __name__ == "__main__":
    main()
