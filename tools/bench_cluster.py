#!/usr/bin/env python3
"""Full-cluster benchmark through the node runtime (control plane + HIP executors),
the analogue of the reference report's experiments (BASELINE.json
configs 3 and 4):

  * two concurrent jobs, AlexNet (500-image queries) and ResNet18 (400-image
    queries), over `--nodes` nodes with the fair-time scheduler;
  * per-model query latency (p50 / mean), whole-cluster images/s, workers per
    query, and the c1/c2 views;
  * optional coordinator kill mid-job (`--kill-coordinator-after S`): the
    standby must promote itself and finish both jobs.

Nodes are in-process over localhost TCP; node i uses cuda:(i % ngpus), so on
a 1-GPU box all nodes share the GPU (throughput is then the single GPU's).

usage: python tools/bench_cluster.py [--nodes 8] [--images 10000] [--kill-coordinator-after 0]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=8)
    ap.add_argument("--images", type=int, default=10000)
    ap.add_argument("--executor", default="hip", choices=["hip", "fake", "torch"])
    ap.add_argument("--kill-coordinator-after", type=float, default=0.0)
    ap.add_argument("--kill-coordinator-at-frac", type=float, default=0.0,
                    help="kill the coordinator once this fraction of both jobs' images is done")
    ap.add_argument("--json", default=None)
    ap.add_argument("--fp32-impl", default="split", choices=["split", "f32mfma"])
    ap.add_argument("--reference-pacing", action="store_true",
                    help="the reference's sleeps: 20 s between a job's queries (:1109), 3 s before each "
                         "chunk (:594), for apples-to-apples query latency (SURVEY.md §7.2 step 7)")
    ap.add_argument("--watchdog", type=float, default=0.0,
                    help="dump every thread's stack and exit after this many seconds (hang diagnosis)")
    a = ap.parse_args()
    if a.watchdog:
        import faulthandler

        faulthandler.dump_traceback_later(a.watchdog, exit=True)
    import logging

    import torch

    logging.basicConfig(level=logging.ERROR)
    from bench_recovery import free_base
    from idunno.runtime.cluster import LocalCluster
    from idunno.runtime.data import SyntheticSource
    from idunno.runtime.executor import FakeExecutor, HipExecutor, TorchExecutor

    ngpu = max(1, torch.cuda.device_count()) if a.executor == "hip" else 1

    def exf(i):
        if a.executor == "hip":
            return HipExecutor(f"cuda:{i % ngpu}", seed=0, fp32_impl=a.fp32_impl)
        if a.executor == "torch":
            return TorchExecutor("cpu")
        return FakeExecutor()

    def srcf(i, node):
        if a.executor == "hip":
            return SyntheticSource(node.cfg.data_seed, f"cuda:{i % ngpu}")
        if a.executor == "torch":
            return SyntheticSource(node.cfg.data_seed, "cpu")
        return None

    c = LocalCluster(num_nodes=a.nodes, transport="tcp", base_port=free_base(a.nodes), executor_factory=exf,
                     source_factory=srcf, heartbeat_period_s=0.3, failure_timeout_s=2.0,
                     metadata_period_s=0.5, rpc_timeout_s=30.0).start()
    if a.reference_pacing:        # after the cluster is up: the warm-up below runs unpaced
        pacing = dict(client_query_interval_s=20.0, worker_start_delay_s=3.0)
    out = {"nodes": a.nodes, "gpus": ngpu, "executor": a.executor, "images_per_job": a.images,
           "fp32_impl": a.fp32_impl}
    try:
        cl = c.client(c.cfg.node_name(a.nodes - 2))
        # warm-up: capture graphs for the chunk sizes the fair-time split will produce
        cl.inference(10 ** 6, 10 ** 6 + 400 * 2 - 1, "resnet18")
        cl.inference(10 ** 6, 10 ** 6 + 500 * 2 - 1, "alexnet")
        cl.wait_idle(600)
        coord = c.coordinator()
        base = {m: coord.state.images_done(m) for m in ("alexnet", "resnet18")}
        if a.reference_pacing:
            for k, v in pacing.items():     # every node reads the cluster's one config object
                setattr(c.cfg, k, v)
            out["pacing"] = pacing
        t0 = time.perf_counter()
        ta = cl.submit_job(0, a.images - 1, "alexnet")
        t_second = time.perf_counter()
        tr = cl.submit_job(0, a.images - 1, "resnet18")
        out["second_job_start_s"] = time.perf_counter() - t_second
        killed = False
        want = {m: base[m] + a.images for m in base}
        out["warmup_images"] = base          # counted in c1 too (the warm-up queries above)
        done_frac, killed_at_frac = 0.0, None
        t_log = time.perf_counter()
        while True:
            if not killed and ((a.kill_coordinator_after and time.perf_counter() - t0 > a.kill_coordinator_after)
                               or (a.kill_coordinator_at_frac and done_frac >= a.kill_coordinator_at_frac)):
                c.crash(c.cfg.coordinator_name)
                killed = True
                t_kill = time.perf_counter()
                killed_at_frac = done_frac
            try:
                s = cl.view("summary")
            except Exception:  # noqa: BLE001  (during failover)
                time.sleep(0.05)
                continue
            if all(s["done"].get(m, 0) >= want[m] for m in want) and s["pending"] == 0:
                break
            done_frac = sum(s["done"].get(m, 0) - base[m] for m in want) / (2 * a.images)
            if time.perf_counter() - t0 > 1800:
                raise TimeoutError(s)
            if time.perf_counter() - t_log > 5:        # progress (and a trail if it stalls)
                t_log = time.perf_counter()
                print(f"[{t_log - t0:7.1f}s] done {s['done']} pending {s['pending']} "
                      f"coordinator {c.coordinator().name}", file=sys.stderr, flush=True)
                if t_log - t0 > (20 if not a.reference_pacing else 600):   # stalled: per-query image coverage
                    st = c.coordinator().state
                    with st.lock:
                        for (m, q), ents in sorted(st.worker_set.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
                            got = sum(b - a + 1 for a, b in st._done_imgs.get((m, q), []))
                            span = (min(e[1] for e in ents), max(e[2] for e in ents)) if ents else None
                            print(f"   {m} q{q} span {span} imgs {got} chunks "
                                  f"{[(e[0], e[1], e[2], e[3]) for e in ents]}", file=sys.stderr, flush=True)
                        print(f"   jobs {st.jobs} next_qnum {dict(st.next_qnum)}", file=sys.stderr, flush=True)
                    raise SystemExit(3)
            time.sleep(0.01)
        wall = time.perf_counter() - t0
        deadline = time.perf_counter() + 30       # a promotion may still be under way
        while True:
            try:
                coord = c.coordinator()
                break
            except RuntimeError:
                if time.perf_counter() > deadline:
                    raise
                time.sleep(0.05)
        lat = {m: coord.state.query_latency.get(m, [])[-(a.images // coord.cfg.batch_for(m)):] for m in want}
        workers = {}
        for (m, q), ents in coord.state.worker_set.items():
            workers.setdefault(m, []).append(len({e[0] for e in ents}))
        out.update({
            "wall_s": round(wall, 3),
            "images_per_s": round(2 * a.images / wall, 1),
            "query_latency_p50_s": {m: round(statistics.median(v), 4) for m, v in lat.items() if v},
            "query_latency_mean_s": {m: round(statistics.mean(v), 4) for m, v in lat.items() if v},
            "workers_per_query_median": {m: statistics.median(v) for m, v in workers.items()},
            "coordinator_killed": killed,
            "final_coordinator": coord.name,
            "c1": cl.view("c1")["text"],
            "c2": cl.view("c2")["text"],
            "job_replies": [ta, tr],
        })
        if killed:
            out["failover_to_done_s"] = round(time.perf_counter() - t_kill, 3)
            out["killed_at_done_fraction"] = round(killed_at_frac, 3)
    finally:
        c.stop()
    print(json.dumps(out, indent=1, default=str))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1, default=str)


if __name__ == "__main__":
    main()
