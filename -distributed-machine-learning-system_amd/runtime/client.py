"""Client API behind the shell (reference ``inference`` / ``send_inference_command``,
mp4_machinelearning.py:947-969, 1104-1109).

``inference(start, end, model)`` cuts ``[start, end]`` into batch-size queries
``[i, min(i + bs - 1, end)]`` (fix A16: the reference's range loop overshot a
non-aligned end) and submits each to the acting coordinator, falling back to
the hot standby when the coordinator is unreachable, with the reference's
inter-query pacing as a knob (``client_query_interval_s``, 20 s in the
reference, 0 by default here).
"""
from __future__ import annotations

import json
import threading
import time

from ..models.reference import canonical
from .messages import Type
from .transport import TransportError


class Client:
    def __init__(self, node):
        self.node = node
        self.cfg = node.cfg
        self.submitted: list[dict] = []
        self.lock = threading.Lock()

    def _call(self, msg: dict, timeout: float | None = None) -> dict:
        timeout = timeout or self.cfg.rpc_timeout_s
        master = self.node.membership.master
        targets = [master] + ([self.cfg.standby_name] if self.cfg.standby_name != master else [])
        last = None
        for dst in targets:
            try:
                if dst == self.node.name:
                    r = self.node.handle(dict(msg, src=self.node.name))
                    if r is not None:
                        return r
                    continue
                return self.node.transport.request(dst, msg, timeout)
            except TransportError as e:
                last = e
        raise TransportError(f"coordinator and standby unreachable: {last}")

    def submit(self, model: str, start: int, end: int) -> dict:
        r = self._call({"t": Type.INFERENCE, "model": model, "start": start, "end": end})
        with self.lock:
            self.submitted.append({"model": model, "start": start, "end": end, "reply": r,
                                   "t": time.time()})
        return r

    def inference(self, start: int, end: int, model: str, interval_s: float | None = None) -> list[dict]:
        model = canonical(model)
        bs = self.cfg.batch_for(model)
        interval = self.cfg.client_query_interval_s if interval_s is None else interval_s
        out = []
        for i in range(start, end + 1, bs):
            out.append(self.submit(model, i, min(i + bs - 1, end)))
            if interval and i + bs <= end:
                time.sleep(interval)
        return out

    def submit_job(self, start: int, end: int, model: str) -> dict:
        """Send the whole range once; the coordinator batches it (C28 variant)."""
        return self._call({"t": Type.INFERENCE, "model": model, "start": start, "end": end, "job": True})

    def inference_async(self, start: int, end: int, model: str) -> threading.Thread:
        th = threading.Thread(target=self.inference, args=(start, end, model), daemon=True)
        th.start()
        return th

    def view(self, name: str) -> dict:
        return self._call({"t": Type.STATS, "view": name})

    def c4(self, path: str = "result.txt") -> dict:
        r = self.view("c4")
        res = r.get("results", {})
        with open(path, "w") as f:
            f.write(json.dumps(res))
        return res

    def wait_idle(self, timeout: float = 30.0, expect_images: dict | None = None) -> dict:
        """Poll the coordinator until nothing is pending (and counts reached)."""
        end = time.monotonic() + timeout
        s = {}
        while time.monotonic() < end:
            try:
                s = self.view("summary")
            except TransportError:
                time.sleep(0.05)
                continue
            ok = s.get("pending", 1) == 0
            if expect_images:
                ok = ok and all(s.get("done", {}).get(m, 0) >= n for m, n in expect_images.items())
            if ok:
                return s
            time.sleep(0.02)
        return s

    def grep(self, pattern: str) -> list[str]:
        lines = []
        for n in self.node.membership.alive():
            try:
                if n == self.node.name:
                    lines += self.node.local_grep(pattern)
                else:
                    lines += self.node.transport.request(n, {"t": Type.GREP, "pattern": pattern},
                                                         self.cfg.rpc_timeout_s).get("lines", [])
            except TransportError:
                lines.append(f"{n}: <unreachable>")
        return lines

    def trace(self, path: str) -> int:
        """Collect every live node's spans into one Chrome trace file."""
        from ..utils.tracing import write_chrome_trace

        lists = []
        for n in self.node.membership.alive():
            try:
                if n == self.node.name:
                    lists.append(self.node.tracer.export())
                else:
                    lists.append(self.node.transport.request(n, {"t": Type.STATS, "view": "trace"},
                                                             self.cfg.rpc_timeout_s).get("events", []))
            except TransportError:
                pass
        return write_chrome_trace(path, lists)

    def checkpoint(self) -> dict:
        return self._call({"t": Type.STATS, "view": "checkpoint"})

    def kill(self, node: str, mode: str = "crash", seconds: float = 1.0) -> bool:
        if node == self.node.name:
            self.node.handle({"t": Type.KILL, "mode": mode, "seconds": seconds, "src": self.node.name})
            return True
        return self.node.transport.send(node, {"t": Type.KILL, "mode": mode, "seconds": seconds})
