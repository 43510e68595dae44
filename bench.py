#!/usr/bin/env python3
"""Headline benchmark: ResNet18 bs=400 image-classification queries on 1..8 MI355X.

Metric (BASELINE.json): images/sec for the whole node + p50 query latency,
ResNet18, 400 images per query per GPU, synthetic 224x224x3 uint8 images and
random-init weights (no datasets or checkpoints are reachable).

Precision: the reference classifies in fp32 (torchvision eager,
/root/reference/alexnet_resnet.py:17-22, 74-75), so the headline runs the
framework's fp32 path (``--fp32-impl``):
  * "split" (default): every conv (the fused stem, the residual stages) on
    fp32-accurate split fp16 -- each fp32 value carried as (hi, lo) halfs (22
    significant bits, 4 bytes like fp32), hi*hi + hi*lo + lo*hi summed in f32
    on the f16 MFMA -- and the FC on the f32-input MFMA;
  * "f32mfma": every conv / FC on v_mfma_f32_16x16x4_f32 (exact f32 products,
    f32 accumulate), 3x3 stride-1 convs by fused fp32 Winograd F(2x2,3x3).
Both are checked against the fp64 CPU module on the same weights, next to
torch fp32 itself (``max_rel_logit_err_vs_fp64``,
``torch_fp32_max_rel_logit_err_vs_fp64``, ``max_rel_logit_err_vs_torch_fp32``).
The other fp32 implementation and the fp16 path (f16 MFMA, f32 accumulate,
fp16 activations) are reported as extra keys.

One *step* is one round of the cluster's query path, end to end:
  1. the coordinator (rank 0) splits the round's image range over the ranks
     with the scheduler's split rule (reference mp4_machinelearning.py:523-536)
     and dispatches the chunk descriptors (RCCL broadcast);
  2. every rank takes its chunk from its HBM-resident replica of the dataset
     and runs preprocess + the HIP forward + fused softmax-top1 (one hipGraph
     replay of hand-written gfx950 kernels, window start read on the device);
  3. top-1 (class, prob) pairs are gathered to the coordinator over RCCL,
     copied to host and recorded in the job-state tables.
Headline = weak scaling (400 images per GPU per step).  Strong scaling (ONE
400-image query split over the N ranks, as the reference splits a query over
its workers) is reported as ``*_strong`` keys.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  --gpus N > 1 without torchrun env vars: bench.py starts N rank processes
  itself (one per GPU, RCCL over 127.0.0.1 rendezvous) and exits non-zero if
  any rank fails.  Under torchrun (RANK set) it is one rank of the job.
  --dry-run: gloo on the CPU with a fake forward (tests the launcher, the
  collectives and the JSON contract without a GPU).
  --system: the same metric through the fault-tolerant cluster runtime: every
  rank runs a Node (membership + failure detector, coordinator on rank 0, hot
  standby on the last rank), rank 0's client submits the queries to the
  coordinator, which schedules them (fair-time split) as RCCL rounds over the
  ranks (N > 1; TCP control plane for N = 1) and ingests the results into the
  job-state tables.  Prints one JSON line with "mode": "system".
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

BASELINE_IMG_PER_S = 41.0          # 400 img / 9.749 s (ResNet18, 5 workers)
BASELINE_P50_S = 9.749             # p50 ResNet18 400-image query latency
METRIC = "images/sec (whole node) + p50 query latency, ResNet18 bs=400 at 1/2/4/8 GPU"
QUERY = 400                        # images per query (reference report p.1, ResNet18)
COMPUTE_F32 = ("f32-input MFMA (v_mfma_f32_16x16x4_f32), fp32 activations/weights, fp32 accumulate; "
               "3x3/s1 convs by fused fp32 Winograd F(2x2,3x3)")
COMPUTE_SPLIT = ("fp32-accurate: every conv (fused stem, residual stages) on split fp16 (each fp32 value as "
                 "hi+lo halfs, 22-bit significand, 4 bytes; hi*hi+hi*lo+lo*hi on v_mfma_f32_16x16x32_f16, "
                 "fp32 accumulate), FC on the f32-input MFMA; logits checked against fp64 next to torch fp32")


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "fp16"],
                    help="headline precision (fp32 = the reference's)")
    ap.add_argument("--fp32-impl", default="split", choices=["split", "f32mfma"],
                    help="fp32 kernels: split-fp16 (fp32-accurate) residual stages, or all f32-MFMA")
    ap.add_argument("--batch", type=int, default=400, help="images per GPU per weak-scaling step")
    ap.add_argument("--dataset-images", type=int, default=2000,
                    help="synthetic images replicated in every rank's HBM (grown to fit a round)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--no-extras", action="store_true", help="skip the strong-scaling / fp16 / numerics extras")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--dry-run", action="store_true", help="CPU + gloo + fake forward (launcher/contract test)")
    ap.add_argument("--fail-rank", type=int, default=-1, help="testing: this rank exits 3 after warmup")
    ap.add_argument("--launch-timeout", type=float, default=1500.0, help="self-launch: seconds before ranks are killed")
    ap.add_argument("--system", action="store_true", help="measure through the node runtime (see docstring)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# self-launch (no torchrun): one child process per GPU, started before any
# HIP call in this process
# ---------------------------------------------------------------------------

def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_local(a, argv) -> int:
    n = a.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    deadline = time.time() + a.launch_timeout
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                print(f"bench: a rank exited with {rc}; stopping the others", file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in codes):
                return 0
            if time.time() > deadline:
                print("bench: ranks timed out", file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc if rc else 1


# ---------------------------------------------------------------------------
# one rank
# ---------------------------------------------------------------------------

class FakeRunner:
    """--dry-run forward: class = global image index % 1000, prob 0.5."""

    def __init__(self, device):
        self.device = device

    def window(self, dataset, batch, start, packed):
        import torch

        def run():
            s = int(start.item())
            idx = torch.arange(s, s + batch, dtype=torch.int32)
            packed[:batch, 0].copy_(idx % 1000)
            packed[:batch, 1].copy_(torch.full((batch,), 0.5).view(torch.int32))
        return run


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "RANK" not in os.environ and a.gpus > 1:
        return launch_local(a, argv)

    if a.system:
        return run_system(a)

    import numpy as np
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from idunno.parallel.dataplane import QueryPlane, init_from_env
    from idunno.runtime.jobstate import JobState
    from idunno.runtime.scheduler import split_range

    env = init_from_env(backend="gloo" if a.dry_run else None, cpu=a.dry_run)
    if env.world != a.gpus:
        print(json.dumps({"error": f"--gpus {a.gpus} but WORLD_SIZE={env.world}"}), flush=True)
        return 2
    if not a.dry_run and env.device.type != "cuda":
        print(json.dumps({"error": "bench.py needs a GPU (MI355X); use --dry-run on CPU"}), flush=True)
        return 2
    gpu = env.device.type == "cuda"
    coord = env.rank == 0
    W = env.world
    B = a.batch
    strong_chunk = -(-QUERY // W)
    # every rank holds a replica of the synthetic dataset (SDFS replication
    # factor = world): any chunk of a query can be served by any rank
    D = max(a.dataset_images, (W + 1) * B)

    def sync():
        if gpu:
            torch.cuda.synchronize()

    def barrier():
        if env.distributed:
            dist.barrier()
        sync()

    if a.dry_run:
        dataset = None
    else:
        from idunno import ops
        dataset = ops.synth_images(a.seed + 1234, 0, D, env.device)

    plane = QueryPlane(env, coordinator=0, max_chunk=max(B, strong_chunk))
    start_dev, send = plane.row_start(), plane.send_buffer
    model_id = 1 if a.model.startswith("resnet") else 0

    def make_run(runner, batch):
        if runner is None:
            return FakeRunner(env.device).window(dataset, batch, start_dev, send)
        if a.no_graph:
            return lambda: runner.forward(dataset, start_dev, batch, 0, send)
        _, run = runner.capture_window(dataset, batch, start=start_dev, start_offset=0, packed=send)
        return run

    def measure(run, per_round: int, steps: int, warmup: int, label: str):
        """Time `steps` pipelined rounds of `per_round` images (split over the
        ranks), then `unloaded` rounds one at a time for the p50 latency."""
        state = JobState() if coord else None
        host = [torch.empty(W, plane.max_chunk, 2, dtype=torch.int32, pin_memory=gpu) for _ in range(2)] \
            if coord else None
        lat, pending = [], []

        def ingest():
            ev, table, slot, t0 = pending.pop(0)
            if ev is not None:
                ev.synchronize()
            t1 = time.perf_counter()
            res = host[slot].numpy()
            cls_all, prob_all = res[:, :, 0], res[:, :, 1].view(np.float32)
            for r, row in enumerate(table):
                n = row[3] - row[2] + 1
                state.record_result(a.model, row[1], f"rank{r}", row[2], row[3], cls_all[r, :n].copy(),
                                    prob_all[r, :n].copy(), t1)
            lat.append(time.perf_counter() - t0)

        def step(q: int):
            t0 = time.perf_counter()
            table = None
            if coord:
                off = (q * per_round) % (D - max(per_round, plane.max_chunk) + 1)
                chunks = split_range(off, off + per_round - 1, W)
                qnum = q
                table = [(model_id, qnum, s, e) for s, e in chunks]
                state.assign(a.model, qnum, [(f"rank{r}", s, e) for r, (s, e) in enumerate(chunks)], t0)
            plane.dispatch_device(table, slot=q)
            if a.fail_rank == env.rank and q == warmup:
                print(f"bench: rank {env.rank} failing on purpose (--fail-rank)", file=sys.stderr, flush=True)
                os._exit(3)
            run()
            plane.gather(None, None)
            if coord:
                slot = q % 2
                host[slot].copy_(plane.gathered_all, non_blocking=gpu)
                ev = None
                if gpu:
                    ev = torch.cuda.Event()
                    ev.record()
                if pending:
                    ingest()
                pending.append((ev, table, slot, t0))

        def drain():
            if coord:
                while pending:
                    ingest()
            barrier()

        for q in range(warmup):
            step(q)
        drain()
        lat.clear()
        t_start = time.perf_counter()
        for q in range(warmup, warmup + steps):
            step(q)
        drain()
        elapsed = time.perf_counter() - t_start
        if env.distributed:
            t = torch.tensor([elapsed], dtype=torch.float64, device=env.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        p50_loaded = statistics.median(lat) if lat else None
        lat.clear()
        for q in range(warmup + steps, warmup + steps + max(5, min(steps, 20))):
            step(q)
            drain()
        p50 = statistics.median(lat) if lat else None
        recorded = state.images_done(a.model) if coord else None
        return {"elapsed": elapsed, "ips": per_round * steps / elapsed, "p50": p50, "p50_loaded": p50_loaded,
                "recorded": recorded, "label": label}

    # ---- headline: weak scaling at the headline precision --------------------
    runner = None
    if not a.dry_run:
        from idunno.models import HipRunner, build_program, program_flops
        runner = HipRunner(build_program(a.model, seed=a.seed, dtype=a.dtype), env.device)
        runner.split = a.fp32_impl == "split"
    head = measure(make_run(runner, B), W * B, a.steps, a.warmup, "weak")
    extras = {}
    if not a.no_extras:
        # strong scaling: ONE 400-image query split over the W ranks
        strong = measure(make_run(runner, strong_chunk), QUERY, a.steps, a.warmup, "strong")
        extras.update({
            "images_per_s_strong": round(strong["ips"], 2),
            "p50_query_latency_strong_s": round(strong["p50"], 6) if strong["p50"] else None,
            "strong_chunk_per_gpu": strong_chunk,
        })
        if not a.dry_run:
            other = "fp16" if a.dtype == "fp32" else "fp32"
            r2 = HipRunner(build_program(a.model, seed=a.seed, dtype=other), env.device)
            m2 = measure(make_run(r2, B), W * B, a.steps, a.warmup, other)
            extras.update({f"value_{other}": round(m2["ips"], 2),
                           f"ms_per_step_{other}": round(1000 * m2["elapsed"] / a.steps, 4),
                           f"p50_query_latency_{other}_s": round(m2["p50"], 6) if m2["p50"] else None})
            del r2
            if a.dtype == "fp32":
                alt = "f32mfma" if a.fp32_impl == "split" else "split"
                runner.split = alt == "split"
                m3 = measure(make_run(runner, B), W * B, a.steps, a.warmup, alt)
                runner.split = a.fp32_impl == "split"
                extras.update({f"value_fp32_{alt}": round(m3["ips"], 2),
                               f"ms_per_step_fp32_{alt}": round(1000 * m3["elapsed"] / a.steps, 4)})
            if coord:
                extras.update(numerics_check(runner, a, env.device))

    if coord:
        ips = head["ips"]
        p50 = head["p50"]
        headline = a.model == "resnet18" and B == QUERY
        out = {
            "metric": METRIC if headline else
            f"images/sec (whole node) + p50 query latency, {a.model} bs={B} at {W} GPU",
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": W,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * head["elapsed"] / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(ips / BASELINE_IMG_PER_S, 2) if headline else None,
            "dtype": "fp32" if a.dry_run else a.dtype,
            "data": "synthetic uint8 224x224x3 images (dataset replicated in every GPU's HBM), random-init weights",
            "config": {"model": a.model, "global_batch": W * B, "seq_len": None, "image_hw": 224,
                       "batch_per_gpu": B, "parallelism": f"dp{W}", "graph": not a.no_graph,
                       "fp32_impl": a.fp32_impl if a.dtype == "fp32" else None,
                       "compute": (COMPUTE_SPLIT if a.fp32_impl == "split" else COMPUTE_F32) if a.dtype == "fp32" else
                       "f16 MFMA, fp16 activations, fp32 accumulate",
                       "dry_run": a.dry_run},
            "p50_query_latency_s": round(p50, 6) if p50 else None,
            "p50_query_latency_loaded_s": round(head["p50_loaded"], 6) if head["p50_loaded"] else None,
            "p50_vs_baseline_speedup": round(BASELINE_P50_S / p50, 1) if p50 and headline else None,
            "results_recorded": head["recorded"],
            **extras,
        }
        if runner is not None:
            out["model_tflops"] = round(program_flops(runner.p) * ips / 1e12, 2)
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if env.distributed:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def run_system(a) -> int:
    """One rank of the --system measurement (see the module docstring)."""
    import tempfile

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from idunno.config import ClusterConfig
    from idunno.runtime.client import Client
    from idunno.runtime.data import SyntheticSource
    from idunno.runtime.executor import FakeExecutor, HipExecutor
    from idunno.runtime.messages import Type
    from idunno.runtime.node import Node
    from idunno.runtime.transport import TcpTransport, wait_for

    rank = int(os.environ.get("RANK", "0"))
    W = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if W != a.gpus:
        print(json.dumps({"error": f"--gpus {a.gpus} but WORLD_SIZE={W}"}), flush=True)
        return 2
    gpu = not a.dry_run and torch.cuda.is_available()
    if not a.dry_run and not gpu:
        print(json.dumps({"error": "bench.py --system needs a GPU (MI355X); use --dry-run on CPU"}), flush=True)
        return 2
    dev = torch.device("cuda", local) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    B = a.batch
    base = int(os.environ.get("MASTER_PORT", "29500")) + 200
    tmp = tempfile.mkdtemp(prefix=f"idunno_bench_r{rank}_")
    cfg = ClusterConfig(num_nodes=W, base_port=base, store_root=tmp, collective_rounds=W > 1, dtype=a.dtype,
                        max_chunk=B, rpc_timeout_s=60.0, worker_budget=W, dataset_size=10 ** 9,
                        batch_size={a.model: W * B}, collective_port_offset=100)
    name = cfg.node_name(rank)
    ex = FakeExecutor() if a.dry_run else HipExecutor(dev, seed=a.seed, dtype=a.dtype)
    node = Node(cfg, name, TcpTransport(name, cfg.address, cfg.address(name)), ex)
    node.source = None if a.dry_run else SyntheticSource(cfg.data_seed, dev)
    if not a.dry_run:
        ex.warmup(a.model, B)                       # capture before the clock starts
    if rank != 0:
        time.sleep(1.0)                             # the coordinator listens first
    node.start(join=True)
    if rank != 0:
        t_end = time.time() + a.launch_timeout
        while node.alive_flag and time.time() < t_end:
            time.sleep(0.2)
        node.stop()
        return 0
    cl = Client(node)
    try:
        assert wait_for(lambda: len(node.membership.alive()) == W, 60), node.membership.table()
        if W > 1:
            assert wait_for(lambda: node.rounds.group.formed and len(node.rounds.group.members) == W, 60)
        per_q = W * B
        nxt = [0]

        def submit(k):
            for _ in range(k):
                s0 = nxt[0]
                nxt[0] += per_q
                cl.submit(a.model, s0, s0 + per_q - 1)

        def done():
            return node.state.images_done(a.model)

        def wait_done(target, timeout=600):
            return wait_for(lambda: done() >= target and node.state.pending_count() == 0, timeout, 0.001)

        submit(a.warmup)
        assert wait_done(nxt[0]), node.state.summary()
        lat0 = len(node.state.query_latency[a.model])
        t0 = time.perf_counter()
        submit(a.steps)
        assert wait_done(nxt[0]), node.state.summary()
        elapsed = time.perf_counter() - t0
        loaded = sorted(node.state.query_latency[a.model][lat0:])
        lat1 = len(node.state.query_latency[a.model])
        for _ in range(max(5, min(a.steps, 20))):   # unloaded: one query at a time
            submit(1)
            assert wait_done(nxt[0])
        unloaded = sorted(node.state.query_latency[a.model][lat1:])
        rounds = node.rounds.rounds_done if node.rounds is not None else 0
        ips = per_q * a.steps / elapsed
        p50 = unloaded[len(unloaded) // 2]
        out = {
            "metric": METRIC if (a.model == "resnet18" and B == QUERY) else
            f"images/sec (whole node) + p50 query latency, {a.model} bs={B} at {W} GPU",
            "value": round(ips, 2), "unit": "images/sec", "n_gpus": W, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(ips / BASELINE_IMG_PER_S, 2) if a.model == "resnet18" and B == QUERY else None,
            "dtype": "fp32" if a.dry_run else a.dtype, "mode": "system",
            "data": "synthetic uint8 224x224x3 images (SyntheticSource on each GPU), random-init weights",
            "config": {"model": a.model, "global_batch": per_q, "seq_len": None, "image_hw": 224,
                       "batch_per_gpu": B, "parallelism": f"dp{W}",
                       "path": ("client -> coordinator Node (membership, standby) -> fair-time split -> "
                                + ("RCCL rounds" if W > 1 else "local JOB queue") + " -> job-state ingest"),
                       "dry_run": a.dry_run},
            "p50_query_latency_s": round(p50, 6),
            "p50_query_latency_loaded_s": round(loaded[len(loaded) // 2], 6) if loaded else None,
            "p50_vs_baseline_speedup": round(BASELINE_P50_S / p50, 1),
            "results_recorded": done(), "collective_rounds": rounds,
        }
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
        return 0
    finally:
        if node.rounds is not None:
            node.rounds.release()                   # members leave the epoch cleanly
        for m in node.membership.alive():
            if m != node.name:
                node.transport.send(m, {"t": Type.KILL})
        time.sleep(0.2)
        node.stop()


def numerics_check(runner, a, device, n: int = 8) -> dict:
    """Max |logit - oracle| / max |oracle| of the benchmarked program on n
    images against the plain PyTorch fp32 module with the same weights."""
    import torch

    from idunno.models import reference as ref

    m = ref.build(ref.canonical(a.model), seed=a.seed).eval().to(device)
    from idunno import ops

    img = ops.synth_images(a.seed + 99, 0, n, device)
    with torch.no_grad():
        want = m(ref.preprocess_u8(img)).float()
        got = runner.logits(img).float()
        # fp64 oracle on the CPU (same weights): the error torch fp32 itself makes is the yardstick
        x64 = ref.preprocess_u8(img.cpu()).double()
        want64 = m.cpu().double()(x64)
    err = ((got - want).abs().max() / want.abs().max()).item()
    agree = (got.argmax(1) == want.argmax(1)).float().mean().item()
    s64 = want64.abs().max()
    err64 = ((got.cpu().double() - want64).abs().max() / s64).item()
    t64 = ((want.cpu().double() - want64).abs().max() / s64).item()
    return {"max_rel_logit_err_vs_torch_fp32": float(f"{err:.3g}"), "top1_agreement_vs_torch_fp32": agree,
            "max_rel_logit_err_vs_fp64": float(f"{err64:.3g}"),
            "torch_fp32_max_rel_logit_err_vs_fp64": float(f"{t64:.3g}")}


if __name__ == "__main__":
    sys.exit(main())
