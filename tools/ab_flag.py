#!/usr/bin/env python3
"""Same-process A/B of a runtime kernel switch of the extension: the whole
forward hipGraph is captured once with ``<setter>(False)`` and once with
``<setter>(True)`` (the flag is read at launch, so each graph keeps its
setting), then the two graphs are timed in interleaved rounds on one device
(cdna_hip_programming §5.4 rule 24).

usage: python tools/ab_flag.py set_conv_stagger [--model resnet18] [--batch 400] [--dtype fp32]
       python tools/ab_flag.py --attr side_down        (a HipRunner attribute instead)
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("setter", nargs="?", default=None)
    ap.add_argument("--attr", default=None, help="HipRunner attribute to switch instead of an extension setter")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--values", default=None, help="with --attr: 'a,b' integer values instead of False,True")
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=9)
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program

    ext = ops.load()
    setter = getattr(ext, a.setter) if a.setter else (lambda flag: None)
    dev = torch.device("cuda")
    prog = build_program(a.model, dtype=a.dtype)
    shard = ops.synth_images(1234, 0, a.batch, dev)
    runs, outs, keep = {}, {}, []
    vals = (False, True) if not a.values else tuple(int(v) for v in a.values.split(","))
    for flag in vals:
        setter(flag)
        r = HipRunner(prog, dev)
        if a.attr:
            setattr(r, a.attr, flag)
        keep.append(r)
        _start, run = r.capture_window(shard, a.batch)
        runs[flag] = run
        cls, prob = run()
        torch.cuda.synchronize()
        outs[flag] = (cls.clone(), prob.clone())
    setter(False)
    v0, v1 = vals
    agree = (outs[v0][0] == outs[v1][0]).float().mean().item()
    dprob = (outs[v0][1] - outs[v1][1]).abs().max().item()
    print(f"{a.setter or a.attr}: top-1 agreement off vs on {agree:.4f}, max |dprob| {dprob:.2e}", flush=True)
    res = {k: [] for k in runs}
    for _ in range(a.rounds):
        for flag, run in runs.items():
            run()
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.iters):
                run()
            t1.record()
            torch.cuda.synchronize()
            res[flag].append(t0.elapsed_time(t1) / a.iters)
    for flag, v in res.items():
        print(f"{a.setter or a.attr}({flag!s:5s}) {a.model} b{a.batch}: median {statistics.median(v):.4f} ms  "
              f"min {min(v):.4f} ms  rounds {[round(x, 4) for x in v]}", flush=True)
    off, on = statistics.median(res[v0]), statistics.median(res[v1])
    print(f"on vs off: {100 * (off / on - 1):+.2f}% throughput", flush=True)


if __name__ == "__main__":
    main()
