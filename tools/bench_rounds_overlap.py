#!/usr/bin/env python3
"""Cross-round overlap experiment: two full-batch query rounds in flight at once,
each a separately captured hipGraph (own activation pool) replayed on its own
stream, vs the same rounds back-to-back on one stream.  Unlike splitting one
batch (tools/bench_streams.py), every kernel keeps its full-batch shape; the
other round's kernels only fill the first round's wave tails and memory-bound
phases.  Interleaved repeats in one process.

usage: python tools/bench_rounds_overlap.py [--model resnet18] [--batch 400] [--iters 40]
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
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--inflight", default="1,2,3")
    a = ap.parse_args()
    from idunno import ops
    from idunno.models import HipRunner, build_program

    dev = torch.device("cuda")
    runner = HipRunner(build_program(a.model), dev)
    B = a.batch
    kmax = max(int(k) for k in a.inflight.split(","))
    shard = ops.synth_images(1234, 0, kmax * B, dev)
    graphs = []
    for k in range(kmax):
        _, run = runner.capture_window(shard[k * B:(k + 1) * B], B)
        graphs.append(run)
    streams = [torch.cuda.Stream(device=dev) for _ in range(kmax)]
    # reference outputs: each graph alone
    ref = []
    for run in graphs:
        c, p = run()
        torch.cuda.synchronize()
        ref.append((c.clone(), p.clone()))

    def steps(k, n):
        """n rounds; round i runs graph i % kmax on stream i % k."""
        main = torch.cuda.current_stream()
        for st in streams[:k]:
            st.wait_stream(main)
        for i in range(n):
            with torch.cuda.stream(streams[i % k]):
                graphs[i % kmax]()
        for st in streams[:k]:
            main.wait_stream(st)

    res = {int(k): [] for k in a.inflight.split(",")}
    for _ in range(a.rounds):
        for k in res:
            steps(k, kmax * 2)
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            steps(k, a.iters)
            t1.record()
            torch.cuda.synchronize()
            res[k].append(t0.elapsed_time(t1) / a.iters)
    ok = all(torch.equal(graphs[i]()[0], ref[i][0]) for i in range(kmax))
    torch.cuda.synchronize()
    base = statistics.median(res[1]) if 1 in res else None
    for k, v in res.items():
        ms = statistics.median(v)
        gain = f"{(base / ms - 1) * 100:+.2f}% vs 1 in flight" if base else ""
        print(f"{a.model} b{B}: {k} round(s) in flight: median {ms:.4f} ms/round "
              f"({B / ms * 1e3:,.0f} img/s) {gain}  all {[round(x, 4) for x in v]}", flush=True)
    print(f"outputs identical after overlap runs: {ok}", flush=True)


if __name__ == "__main__":
    main()
