#!/usr/bin/env python3
"""Same-process whole-graph A/B of kernel routes: one HipRunner per route
(``HipRunner.route`` bits: 1 no band 3x3, 2 no row-streaming 64->64, 4 no
streaming 1x1), hipGraph replays interleaved round by round on one device.

usage: python tools/ab_route.py [--model resnet50] [--dtype fp16] [--batch 1024] [--routes 0,1]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--routes", default="0,1")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program

    dev = torch.device("cuda")
    ops.load()
    prog = build_program(a.model, dtype=a.dtype)
    shard = ops.synth_images(1234, 0, a.batch, dev)
    runs, outs, keep = {}, {}, []
    for rt in [int(r) for r in a.routes.split(",")]:
        r = HipRunner(prog, dev)
        r.route = rt
        keep.append(r)
        _s, run = r.capture_window(shard, a.batch)
        runs[rt] = run
        cls, prob = run()
        torch.cuda.synchronize()
        outs[rt] = (cls.clone(), prob.clone())
    base = next(iter(outs))
    for rt, (c, p) in outs.items():
        print(f"route {rt}: top-1 agreement vs route {base} {(c == outs[base][0]).float().mean().item():.4f}, "
              f"max |dprob| {(p - outs[base][1]).abs().max().item():.2e}", flush=True)
    res = {k: [] for k in runs}
    for _ in range(a.rounds):
        for rt, run in runs.items():
            run()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(a.iters):
                run()
            en.record()
            torch.cuda.synchronize()
            res[rt].append(st.elapsed_time(en) / a.iters)
    med = {k: statistics.median(v) for k, v in res.items()}
    for rt, v in res.items():
        print(f"route {rt} {a.model} b{a.batch} {a.dtype}: median {med[rt]:.4f} ms  min {min(v):.4f} ms  "
              f"{a.batch / med[rt] * 1e3:.0f} img/s  rounds {[round(x, 4) for x in v]}", flush=True)
    ks = list(med)
    for rt in ks[1:]:
        print(f"route {ks[0]} vs route {rt}: {100 * (med[rt] / med[ks[0]] - 1):+.2f}% throughput", flush=True)


if __name__ == "__main__":
    main()
