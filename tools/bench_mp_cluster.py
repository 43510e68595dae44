#!/usr/bin/env python3
"""Multi-process cluster benchmarks on one host: every node is its own OS
process (``python -m idunno.launch node``) with the HIP executor and the SDFS
image source, as on an MI355X node; failures are real SIGKILLs.

Scenarios (run in order on one cluster; ``--scenarios``):
  overlap     : a cold-cache job over the SDFS dataset; reports the job wall
                time and, from the Chrome trace of every node, how much of each
                prefetched ``chunk.stage`` ran while that node's previous
                ``chunk.compute`` was running (SURVEY.md §2.7 double-buffered
                staging).  Run once with IDUNNO_PREFETCH=1 and once with 0 for
                the A/B (``--prefetch``).
  worker:N    : N queries in flight on a slowed-down worker, which is then
                SIGKILLed; time from the kill until all N queries are answered
                (reference report Fig 4: 5.7 s for 1 task .. 26.8 s for 8).
  coord:N     : N queries in flight when the coordinator process is SIGKILLed;
                time until the hot standby (this process) has promoted itself
                and answered all of them (reference Fig 5: 7.0 s .. 14.0 s).
Every worker scenario kills a different worker; a coord scenario must be last.

usage: python tools/bench_mp_cluster.py --nodes 8 --scenarios overlap,worker:1,worker:4,coord:1 \
           --json out.json [--trace out_trace.json] [--prefetch 0|1]
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REF_WORKER = {1: 5.725, 2: 8.661, 4: 13.425, 6: 19.125, 8: 26.751}
REF_COORD = {1: 6.999, 2: 7.980, 4: 9.977, 6: 11.995, 8: 13.973}


def base_port(n):
    for _ in range(100):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p + n + 700 > 65000:
            continue
        ok = True
        for i in list(range(n)) + [500 + i for i in range(n)]:
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", p + i))
            except OSError:
                ok = False
            finally:
                t.close()
        if ok:
            return p
    raise RuntimeError("no free port range")


def overlap_stats(events):
    """Per node: prefetched stage spans and the share of their time that ran
    under a compute span of the same node."""
    by = {}
    for e in events:
        if e.get("ph") != "X":
            continue
        by.setdefault(e["pid"], []).append(e)
    tot_stage = tot_cover = 0.0
    n_pf = n_pf_overlap = 0
    for evs in by.values():
        comp = [(e["ts"], e["ts"] + e["dur"]) for e in evs if e["name"] == "chunk.compute"]
        for e in evs:
            if e["name"] != "chunk.stage" or not e["args"].get("prefetch"):
                continue
            a, b = e["ts"], e["ts"] + e["dur"]
            cov = sum(max(0.0, min(b, y) - max(a, x)) for x, y in comp)
            n_pf += 1
            n_pf_overlap += cov > 0
            tot_stage += b - a
            tot_cover += min(cov, b - a)
    return {"prefetched_stages": n_pf, "prefetched_stages_overlapping_compute": n_pf_overlap,
            "prefetched_stage_ms": round(tot_stage / 1e3, 3),
            "of_which_under_compute_ms": round(tot_cover / 1e3, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=8)
    ap.add_argument("--scenarios", default="overlap,worker:1,worker:4,coord:1")
    ap.add_argument("--images", type=int, default=4000, help="SDFS dataset size (500-image shards)")
    ap.add_argument("--prefetch", type=int, default=1)
    ap.add_argument("--peer-copy", type=int, default=1, help="SDFS shards GPU-to-GPU from HBM holders (IPC)")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--json", default=None)
    ap.add_argument("--trace", default=None)
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--executor", default="hip", choices=["hip", "fake"], help="fake: CPU dry run")
    a = ap.parse_args()

    import logging

    import torch

    from idunno.config import ClusterConfig
    from idunno.runtime.client import Client
    from idunno.runtime.data import SdfsSource, put_synthetic_dataset
    from idunno.runtime.executor import make_executor
    from idunno.runtime.node import Node
    from idunno.runtime.transport import TcpTransport, wait_for

    logging.basicConfig(level=logging.ERROR)
    n = a.nodes
    base = base_port(n)
    tmp = tempfile.mkdtemp(prefix="idunno_mpc_")
    log_dir = a.log_dir or tmp
    env = dict(os.environ, PYTHONPATH=ROOT, IDUNNO_PREFETCH=str(a.prefetch), IDUNNO_DTYPE=a.dtype,
               IDUNNO_SDFS_PEER_COPY=str(a.peer_copy),
               IDUNNO_METADATA_PERIOD_S="0.2", IDUNNO_RPC_TIMEOUT_S="10", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cfg = ClusterConfig.load(env=env, num_nodes=n, base_port=base, store_root=tmp)
    procs = {}
    t_launch = time.perf_counter()
    for i in range(n - 1):
        err = open(os.path.join(log_dir, f"node{i:02d}.stderr"), "w")
        procs[i] = subprocess.Popen(
            [sys.executable, "-m", "idunno.launch", "node", "--index", str(i), "--nodes", str(n),
             "--base-port", str(base), "--store-root", tmp, "--executor", a.executor, "--source", "sdfs",
             "--join-delay", "2.0"],
            cwd=ROOT, env=env, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=err)
    if a.executor == "hip":
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    me_name = cfg.node_name(n - 1)
    me = Node(cfg, me_name, TcpTransport(me_name, cfg.address, cfg.address(me_name)),
              make_executor(a.executor, dev if a.executor == "hip" else None, seed=cfg.model_seed, dtype=cfg.dtype))
    me.source = SdfsSource(me.sdfs, dev, peer_copy=bool(a.peer_copy))
    out = {"nodes": n, "processes": n, "executor": f"{a.executor} {cfg.dtype}", "gpus": torch.cuda.device_count(),
           "detector": f"{cfg.heartbeat_period_s}s/{cfg.failure_timeout_s}s", "prefetch": bool(a.prefetch), "sdfs_peer_copy": bool(a.peer_copy),
           "kill": "SIGKILL of the node's OS process", "data": f"synthetic uint8 224x224 in SDFS ({a.images} images)"}
    victims = iter(range(2, n - 1))
    cl = Client(me)
    model = "resnet18"
    done_expect = 0

    try:
        time.sleep(3.0)
        me.start(join=True)
        if not wait_for(lambda: len(me.membership.alive()) == n, 240, 0.2):
            raise RuntimeError(f"cluster did not form: {me.membership.table()}")
        out["cluster_up_s"] = round(time.perf_counter() - t_launch, 2)
        t0 = time.perf_counter()
        put_synthetic_dataset(me.sdfs, a.images, cfg.data_seed)
        out["sdfs_put_s"] = round(time.perf_counter() - t0, 2)
        # warm every node's graphs for the per-node chunk size (images beyond the
        # measured range; their shards are fetched now, the measured ones are not)
        bs = cfg.batch_for(model)
        warm0 = a.images - bs
        cl.inference(warm0, a.images - 1, model)
        s = cl.wait_idle(300, {model: bs})
        done_expect = bs
        assert s.get("done", {}).get(model, 0) >= bs, s
        for sc in a.scenarios.split(","):
            kind, _, arg = sc.partition(":")
            if kind == "overlap":
                hi = warm0 - 1
                t0 = time.perf_counter()
                cl.inference(0, hi, model)
                done_expect += hi + 1
                s = cl.wait_idle(600, {model: done_expect})
                wall = time.perf_counter() - t0
                tr = a.trace or os.path.join(tmp, "trace.json")
                cl.trace(tr)
                with open(tr) as f:
                    evs = [e for e in json.load(f)["traceEvents"] if e["ts"] >= (time.time() - wall - 1) * 1e6]
                out["overlap"] = dict(images=hi + 1, wall_s=round(wall, 3), images_per_s=round((hi + 1) / wall, 1),
                                      **overlap_stats(evs))
                print("overlap", out["overlap"], flush=True)
            elif kind == "worker":
                k = int(arg)
                victim = next(victims)
                vname = cfg.node_name(victim)
                cl.kill(vname, "delay", 30.0)           # its chunks queue up behind a 30 s sleep
                time.sleep(0.3)
                for q in range(k):                       # any dataset images (answers are per query)
                    q0 = (q * bs) % (a.images - bs)
                    cl.submit(model, q0, q0 + bs - 1)
                done_expect += k * bs
                time.sleep(1.0)                          # every other chunk answered; the victim holds k
                t0 = time.perf_counter()
                procs[victim].send_signal(signal.SIGKILL)
                s = cl.wait_idle(120, {model: done_expect})
                dt = time.perf_counter() - t0
                ok = s.get("done", {}).get(model, 0) >= done_expect and s.get("pending", 1) == 0
                out.setdefault("worker_failure_s", {})[k] = round(dt, 3) if ok else None
                print(f"worker failure, {k} queries in flight: resumed in {dt:.3f}s (ref {REF_WORKER.get(k)}s)"
                      f" ok={ok}", flush=True)
            elif kind == "coord":
                k = int(arg)
                for nd in me.membership.alive():
                    cl.kill(nd, "delay", 1.5)              # queries still running when the coordinator dies
                for q in range(k):
                    q0 = (q * bs) % (a.images - bs)
                    cl.submit(model, q0, q0 + bs - 1)
                done_expect += k * bs
                time.sleep(0.5)
                t0 = time.perf_counter()
                procs[cfg.coordinator].send_signal(signal.SIGKILL)
                for nd in me.membership.alive():
                    if nd != cfg.coordinator_name:
                        cl.kill(nd, "delay", 0.0)
                ok = wait_for(lambda: me.is_coordinator, 60, 0.01)
                t_promote = time.perf_counter() - t0
                s = cl.wait_idle(120, {model: done_expect})
                dt = time.perf_counter() - t0
                ok = ok and s.get("done", {}).get(model, 0) >= done_expect and s.get("pending", 1) == 0
                out.setdefault("coordinator_failure_s", {})[k] = round(dt, 3) if ok else None
                out.setdefault("standby_promoted_after_s", {})[k] = round(t_promote, 3)
                print(f"coordinator failure, {k} queries in flight: all answered {dt:.3f}s after the kill "
                      f"(promotion {t_promote:.3f}s; ref {REF_COORD.get(k)}s) ok={ok}", flush=True)
                break
        out["reference_worker_failure_s"] = REF_WORKER
        out["reference_coordinator_failure_s"] = REF_COORD
        print(json.dumps(out), flush=True)
        if a.json:
            with open(a.json, "w") as f:
                json.dump(out, f, indent=1)
    finally:
        me.stop()
        for p in procs.values():
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs.values():
            try:
                p.wait(20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait(10)


if __name__ == "__main__":
    main()
