#!/usr/bin/env python3
"""Recovery-time benchmarks, analogues of the reference report's Fig 4 / Fig 5
(BASELINE.md):

  worker   : a worker holding n in-flight chunks is killed; time from the kill
             until every one of those chunks has a result at the coordinator
             (reference: 5.7 s for 1 task ... 26.8 s for 8 tasks);
  coordinator: the coordinator is killed with q queries undone; time from the
             kill until all q queries are complete via the promoted standby
             (reference: 7.0 s for 1 query ... 14.0 s for 8).

Runs N in-process nodes over real localhost TCP.  --executor hip runs the
real GPU path (all nodes share cuda:0 on a 1-GPU box); fake runs on CPU.
The failure detector uses the reference's 0.3 s heartbeat / 2 s timeout by
default (--fast for 0.05 s / 0.3 s).

usage: python tools/bench_recovery.py [--executor fake|hip] [--nodes 8] [--fast]
"""
import argparse
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_base(n):
    for _ in range(100):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        ok = True
        for i in range(n):
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", p + i))
            except OSError:
                ok = False
            finally:
                t.close()
        if ok:
            return p
    raise RuntimeError("no ports")


def make_cluster(a):
    from idunno.runtime.cluster import LocalCluster
    from idunno.runtime.data import SyntheticSource
    from idunno.runtime.executor import FakeExecutor, HipExecutor

    hb, to = (0.05, 0.3) if a.fast else (0.3, 2.0)
    if a.executor == "hip":
        exf = lambda i: HipExecutor("cuda", seed=0)  # noqa: E731
        srcf = lambda i, node: SyntheticSource(node.cfg.data_seed, "cuda")  # noqa: E731
    else:
        exf = lambda i: FakeExecutor(delay_per_image_s=a.fake_delay)  # noqa: E731
        srcf = lambda i, node: None  # noqa: E731
    return LocalCluster(num_nodes=a.nodes, transport="tcp", base_port=free_base(a.nodes), executor_factory=exf,
                        source_factory=srcf, heartbeat_period_s=hb, failure_timeout_s=to,
                        metadata_period_s=0.2, rpc_timeout_s=10.0).start()


def worker_failure(a, ntasks):
    from idunno.runtime.transport import wait_for

    c = make_cluster(a)
    try:
        cl = c.client(c.cfg.node_name(1))
        if a.executor == "hip":   # warm every node's graphs for the chunk size
            cl.inference(0, 80 * a.nodes - 1, "resnet18")
            cl.wait_idle(300, {"resnet18": 80 * a.nodes})
        victim = c.cfg.node_name(2)
        c.nodes[victim].extra_delay_s = 5.0        # chunks queue up on the victim
        coord = c.coordinator()
        base = coord.state.images_done("resnet18")
        # ntasks queries of 80 images, each query split over all nodes -> 1 chunk per node per query
        for q in range(ntasks):
            coord.submit_query("resnet18", 100000 + q * 80 * a.nodes, 100000 + (q + 1) * 80 * a.nodes - 1)
        assert wait_for(lambda: len(coord.state.chunks_of(victim)) == ntasks, 10)
        for n in c.nodes.values():
            if n.name != victim:
                n.extra_delay_s = 0.0
        total = base + ntasks * 80 * a.nodes
        t0 = time.perf_counter()
        c.crash(victim)
        ok = wait_for(lambda: coord.state.images_done("resnet18") >= total, 120, 0.005)
        return time.perf_counter() - t0 if ok else None
    finally:
        c.stop()


def coordinator_failure(a, nq):
    from idunno.runtime.transport import wait_for

    c = make_cluster(a)
    try:
        client = c.client(c.cfg.node_name(a.nodes - 2))
        if a.executor == "hip":
            client.inference(0, 80 * (a.nodes - 1) - 1, "resnet18")
            client.wait_idle(300)
        for n in c.nodes.values():
            n.extra_delay_s = 1.0                   # queries are still running when the coordinator dies
        for q in range(nq):
            client.submit("resnet18", 200000 + q * 400, 200000 + q * 400 + 399)
        time.sleep(0.3)
        for n in c.nodes.values():
            n.extra_delay_s = 0.0
        standby = c.nodes[c.cfg.standby_name]
        t0 = time.perf_counter()
        c.crash(c.cfg.coordinator_name)
        need = standby.state.images_done("resnet18")
        ok = wait_for(lambda: standby.is_coordinator and not standby.state.pending() and
                      all(standby.state.finished_queries.get("resnet18", 0) >= 0 for _ in [0]), 120, 0.005)
        # every image of the nq undone queries must be answered
        want = {i for q in range(nq) for i in range(200000 + q * 400, 200000 + q * 400 + 400)}
        ok = ok and wait_for(lambda: want <= {s + k for ch in sum((v for v in standby.state.results.values()), [])
                                              for s in [ch.start] for k in range(ch.end - ch.start + 1)}, 120, 0.01)
        del need
        return time.perf_counter() - t0 if ok else None
    finally:
        c.stop()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--executor", default="fake", choices=["fake", "hip"])
    ap.add_argument("--nodes", type=int, default=8)
    ap.add_argument("--fast", action="store_true")
    ap.add_argument("--fake-delay", type=float, default=0.0)
    ap.add_argument("--tasks", default="1,2,4,6,8")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import logging

    logging.basicConfig(level=logging.ERROR)
    out = {"executor": a.executor, "nodes": a.nodes, "detector": "0.05s/0.3s" if a.fast else "0.3s/2s",
           "worker_failure_s": {}, "coordinator_failure_s": {}}
    ref_w = {1: 5.725, 2: 8.661, 4: 13.425, 6: 19.125, 8: 26.751}
    ref_c = {1: 6.999, 2: 7.980, 4: 9.977, 6: 11.995, 8: 13.973}
    for n in [int(x) for x in a.tasks.split(",")]:
        tw = worker_failure(a, n)
        tc = coordinator_failure(a, n)
        out["worker_failure_s"][n] = tw
        out["coordinator_failure_s"][n] = tc
        print(f"n={n}: worker-failure resume {tw:.3f}s (ref {ref_w.get(n)}s)  "
              f"coordinator-failure recovery {tc:.3f}s (ref {ref_c.get(n)}s)", flush=True)
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
