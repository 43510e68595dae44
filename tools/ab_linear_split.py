#!/usr/bin/env python3
"""Same-process A/B of split-K FC layers: the whole forward graph captured with
every FC layer split into each of the given K-split counts (ops.LINEAR_SPLITS).

usage: python tools/ab_linear_split.py [--model alexnet] [--batch 500]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--batch", type=int, default=500)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--variants", default="1,auto", help="split counts forced on every FC layer ('auto': ops heuristic)")
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program

    dev = torch.device("cuda")
    prog = build_program(a.model)
    shard = ops.synth_images(1234, 0, a.batch, dev)
    runs, outs, keep = {}, {}, []
    variants = [(v, None if v == "auto" else int(v)) for v in a.variants.split(",")]
    for name, forced in variants:
        ops.LINEAR_SPLITS = forced
        r = HipRunner(prog, dev)
        keep.append(r)
        _s, run = r.capture_window(shard, a.batch)
        runs[name] = run
        c, p = run()
        torch.cuda.synchronize()
        outs[name] = (c.clone(), p.clone())
    ops.LINEAR_SPLITS = None
    first = variants[0][0]
    for name in runs:
        agree = (outs[first][0] == outs[name][0]).float().mean().item()
        print(f"{name} vs {first}: top-1 agreement {agree:.4f}, "
              f"max |dprob| {(outs[first][1] - outs[name][1]).abs().max().item():.2e}")
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
    base = statistics.median(res[first])
    for name, v in res.items():
        m = statistics.median(v)
        print(f"{a.model} b{a.batch} {name:8s}: median {m:.4f} ms ({a.batch / m * 1e3:,.0f} img/s, "
              f"{100 * (base / m - 1):+.2f}%)  rounds {[round(x, 4) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
