#!/usr/bin/env python3
"""Concurrency experiment: one 400-image query per step, forward split into
S sub-batches whose hipGraphs replay on S streams at once, so one branch's
memory-bound phases (stem, layer1) and kernel tails overlap the other's
compute-bound layers.  Interleaved rounds in one process (rule 24).

usage: python tools/bench_streams.py [--model resnet18] [--batch 400] [--iters 30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=400)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--dtype", default="fp16", help="fp16, or fp32 (split fp16, the headline)")
    ap.add_argument("--queries", action="store_true",
                    help="S whole queries (S graphs of --batch images) on S streams per step, not S sub-batches")
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program

    dev = torch.device("cuda")
    runner = HipRunner(build_program(a.model, dtype=a.dtype), dev)
    shard = ops.synth_images(1234, 0, 5 * a.batch, dev)
    cfgs = {}
    for S in [int(s) for s in a.splits.split(",")]:
        n = a.batch if a.queries else a.batch // S
        streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
        # graph k reads images [k*n, (k+1)*n) of the shard (distinct views -> distinct graphs)
        graphs = []
        for k in range(S):
            start, run = runner.capture_window(shard[k * n:], n)
            graphs.append(run)
        cfgs[S] = (streams, graphs)

    def step(S):
        streams, graphs = cfgs[S]
        main = torch.cuda.current_stream()
        for st, run in zip(streams, graphs):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                run()
        for st in streams:
            main.wait_stream(st)

    res = {S: [] for S in cfgs}
    for _ in range(a.rounds):
        for S in cfgs:
            step(S)
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.iters):
                step(S)
            t1.record()
            torch.cuda.synchronize()
            res[S].append(t0.elapsed_time(t1) / a.iters)
    for S, v in res.items():
        ms = min(v)
        imgs = a.batch * S if a.queries else a.batch
        what = f"{S} queries of {a.batch}" if a.queries else f"{S} x {a.batch // S}"
        print(f"{a.model} batch {a.batch} as {what} on {S} streams: {ms:.3f} ms/step "
              f"({imgs / ms * 1e3:,.0f} img/s)  all rounds {[round(x, 3) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
