#!/usr/bin/env python3
"""Front split experiment: the whole forward hipGraph with the stem + layer1
run on S batch parts (activations of one part stay in the 256 MiB Infinity
Cache) vs S = 1, interleaved rounds in one process.  Also checks that every
split gives bit-identical results.

usage: python tools/bench_split.py [--model resnet18] [--batch 400] [--splits 1,2,4]
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
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--splits", default="1,2,4")
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program

    dev = torch.device("cuda")
    prog = build_program(a.model)
    shard = ops.synth_images(1234, 0, a.batch + 16, dev)
    runs, outs, keep = {}, {}, []
    for S in [int(x) for x in a.splits.split(",")]:
        r = HipRunner(prog, dev, front_split=S)
        keep.append(r)
        start, run = r.capture_window(shard, a.batch)
        start.fill_(7)
        runs[S] = run
        cls, prob = run()
        torch.cuda.synchronize()
        outs[S] = (cls.clone(), prob.clone())
    base = min(outs)
    for S, (c, p) in outs.items():
        print(f"split {S}: identical to split {base}: {bool(torch.equal(c, outs[base][0]) and torch.equal(p, outs[base][1]))}",
              flush=True)
    res = {k: [] for k in runs}
    for _ in range(a.rounds):
        for S, run in runs.items():
            run()
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.iters):
                run()
            t1.record()
            torch.cuda.synchronize()
            res[S].append(t0.elapsed_time(t1) / a.iters)
    m1 = statistics.median(res[base])
    for S, v in res.items():
        m = statistics.median(v)
        print(f"{a.model} b{a.batch} front_split {S}: median {m:.4f} ms ({a.batch / m * 1e3:,.0f} img/s, "
              f"{100 * (m1 / m - 1):+.2f}% vs split {base})  rounds {[round(x, 4) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
