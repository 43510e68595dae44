#!/usr/bin/env python3
"""Coordinator host cost of one collective round, in isolation (no process
group, no other processes competing for the CPU): the job-state assignment of a
400-image query over W members plus ``RoundPlane._finalize`` of its gathered
round (header read, scheduler feedback, vectorised ingest).  VERDICT r5 item 6.

    python tools/hostcost_probe.py [--members 1 8] [--rounds 2000]
"""
from __future__ import annotations

import argparse
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from idunno.config import ClusterConfig  # noqa: E402
from idunno.parallel.elastic import HDR_ROWS  # noqa: E402
from idunno.runtime.jobstate import JobState  # noqa: E402
from idunno.runtime.rounds import RoundPlane, _Query, _Round  # noqa: E402
from idunno.runtime.scheduler import FairTimeScheduler, split_range  # noqa: E402


class _Tracer:
    def instant(self, *a, **k):
        pass


class _Membership:
    def is_alive(self, m):
        return True


class _Node:
    def __init__(self, members):
        self.name = members[0]
        self.standby = members[-1]
        self.cfg = ClusterConfig()
        self.state = JobState(batchsize={"resnet18": 400})
        self.sched = FairTimeScheduler(budget=len(members))
        self.tracer = _Tracer()
        self.membership = _Membership()
        self._progress = threading.Condition()

    def _ingest_round(self, recs, now, seq=-1):
        new = self.state.record_results(recs, now)
        if new:
            with self._progress:
                self._progress.notify_all()
        return new


class _Group:
    def __init__(self, world, max_chunk):
        self.max_chunk = max_chunk
        self.standby_rank = world - 1 if world > 1 else -1
        self.arr = np.zeros((world, max_chunk + HDR_ROWS, 2), np.int32)
        self.arr[:, max_chunk, :] = [900, 1]          # (us, model id)
        self.arr[:, max_chunk + 1, :] = [50, 0]       # (n, tag)

    def collect(self, seq, work, check=None):
        return self.arr

    def release(self, work, check=None):
        pass


def probe(world: int, rounds: int) -> float:
    members = tuple(f"node{i:02d}" for i in range(world))
    node = _Node(members)
    plane = RoundPlane.__new__(RoundPlane)
    plane.node, plane.cfg = node, node.cfg
    plane.group = _Group(world, 512)
    plane.rounds_done = 0
    plane.host_s = plane.host_cpu_s = plane.host_wait_s = 0.0
    plane._mirror_q = None
    t_total = 0.0
    for q in range(rounds):
        s0 = q * 400
        plan = [(w, s, e) for w, (s, e) in zip(members, split_range(s0, s0 + 399, world))]
        t0 = time.perf_counter()
        node.state.assign("resnet18", q, plan, time.time())
        qq = _Query("resnet18", q, {w: (s, e) for w, s, e in plan}, members)
        r = _Round(q, [qq], RoundPlane._table(members, [qq]))
        plane._finalize(r, members, None)
        t_total += time.perf_counter() - t0
    return 1000 * t_total / rounds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--members", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--rounds", type=int, default=2000)
    a = ap.parse_args()
    for w in a.members:
        probe(w, 200)                                  # warm
        ms = min(probe(w, a.rounds) for _ in range(3))
        print(f"members {w}: {ms * 1000:.1f} us per round (assign + finalize)", flush=True)


if __name__ == "__main__":
    main()
