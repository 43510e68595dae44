"""Per-query span tracing ("per-query spans: submit -> dispatch
-> stage -> compute -> gather -> result").  The reference has only DEBUG prints.

Every node owns a ``Tracer``; spans are recorded with wall-clock timestamps
(all nodes of one host share the clock) and exported as Chrome trace-event JSON
(open in chrome://tracing or Perfetto), one process row per node.  Recording is
a deque append under a lock; the ring is bounded so tracing can stay on.
"""
from __future__ import annotations

import json
import threading
import time
from collections import deque
from contextlib import contextmanager


class Tracer:
    def __init__(self, node: str, capacity: int = 100_000, enabled: bool = True):
        self.node = node
        self.enabled = enabled
        self.events: deque = deque(maxlen=capacity)
        self.lock = threading.Lock()

    def instant(self, name: str, **args) -> None:
        if self.enabled:
            with self.lock:
                self.events.append(("i", name, time.time(), 0.0, args, threading.get_ident()))

    def complete(self, name: str, t0: float, t1: float, **args) -> None:
        if self.enabled:
            with self.lock:
                self.events.append(("X", name, t0, t1 - t0, args, threading.get_ident()))

    @contextmanager
    def span(self, name: str, **args):
        t0 = time.time()
        try:
            yield
        finally:
            self.complete(name, t0, time.time(), **args)

    def export(self) -> list[dict]:
        with self.lock:
            evs = list(self.events)
        out = []
        for ph, name, ts, dur, args, tid in evs:
            e = {"name": name, "ph": ph, "ts": ts * 1e6, "pid": self.node, "tid": tid % 100000, "args": args}
            if ph == "X":
                e["dur"] = dur * 1e6
            else:
                e["s"] = "t"
            out.append(e)
        return out


def write_chrome_trace(path: str, event_lists: list[list[dict]]) -> int:
    evs = [e for lst in event_lists for e in lst]
    with open(path, "w") as f:
        json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)
    return len(evs)
