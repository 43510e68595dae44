"""Collective query rounds inside the fault-tolerant node runtime.

When ``cfg.collective_rounds`` is on (one node per process, e.g. one per GPU
via ``idunno.launch``), a query whose plan puts at most one chunk on each
group member runs as ONE collective round on the ``ElasticGroup`` (RCCL
broadcast of the descriptor table + gather of packed top-1 results, the same
``QueryPlane`` bench.py drives) instead of per-chunk TCP JOB/RESULT messages.
The reference has no equivalent (every chunk is a TCP message,
mp4_machinelearning.py:560-613); the TCP path stays as the fallback:

  * a round whose collectives fail is abandoned and its chunks are re-sent as
    TCP JOBs (results are idempotent by chunk key);
  * every membership change (failure, join, standby promotion) makes the
    coordinator re-form the group under a new epoch over the live members.

Each node runs ONE driver thread that owns the process group, so forming,
rounds and teardown never race: as coordinator it forms epochs and serves the
round queue, as a member it follows the latest GROUP_FORM it was sent.

Liveness: collectives are polled against the failure
detector, never waited on blindly.  The coordinator abandons a round as soon
as membership marks one of its members dead (``failure_timeout_s``), falls
back to TCP for the live members' chunks and aborts the epoch in the
background; a member abandons its wait when a newer epoch is announced or
the coordinator is dead.  Idle gaps are free (the process-group timeout is
long), so no keepalive rounds are needed.

Results stay on the device: a member's forward writes its packed top-1 pairs
straight into the gather's send buffer (``HipExecutor.run_packed``), and the
coordinator copies the whole round to the host once.
"""
from __future__ import annotations

import logging
import queue
import threading
import time

import numpy as np

from ..parallel.dataplane import NO_WORK
from ..parallel.elastic import MODEL_IDS, STOP, ElasticGroup, RoundAbandoned
from .messages import Type

log = logging.getLogger("idunno.rounds")


class RoundPlane:
    def __init__(self, node, device):
        self.node = node
        self.cfg = node.cfg
        self.group = ElasticGroup(device, timeout_s=self.cfg.collective_timeout_s, max_chunk=self.cfg.max_chunk)
        self.q: queue.Queue = queue.Queue()
        self.lock = threading.Lock()
        self.epoch = 0                      # last epoch formed or announced
        self.members: list[str] = []
        self.healthy = False                # coordinator: rounds may be queued
        self.rounds_done = 0
        self.rounds_failed = 0
        self._reform_at: float | None = None
        self._pending_form: dict | None = None
        self._released = False
        self._wake = threading.Event()
        self._thread: threading.Thread | None = None

    def start(self) -> None:
        self._thread = threading.Thread(target=self._driver, name=f"{self.node.name}-rounds", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._wake.set()

    def join(self, timeout: float = 5.0) -> None:
        """Wait for the driver thread and any background epoch abort to end
        (a process must not exit while a communicator is being torn down)."""
        th = self._thread
        if th is not None and th is not threading.current_thread():
            th.join(timeout)
        self.group._join_aborter(timeout)

    def release(self, timeout: float = 10.0) -> bool:
        """Coordinator: end the epoch cleanly (a STOP round lets every member
        leave its round loop and destroy the group) and form no new one.
        Used before a planned shutdown of the whole cluster."""
        done = threading.Event()
        with self.lock:
            self.healthy = False
            self._released = True
        self.q.put(("__release__", done))
        self._wake.set()
        return done.wait(timeout)

    # -- triggers (any thread) ----------------------------------------------------------
    def schedule_reform(self, reason: str, delay: float = 0.2) -> None:
        """Coordinator: re-form the group over the live members after ``delay``
        (several triggers inside the window collapse into one re-form)."""
        with self.lock:
            self.healthy = False
            at = time.monotonic() + delay
            self._reform_at = at if self._reform_at is None else min(self._reform_at, at)
        log.info("%s: re-form scheduled (%s)", self.node.name, reason)
        self._wake.set()

    def on_group_form(self, msg: dict) -> None:
        with self.lock:
            if int(msg["epoch"]) <= self.epoch:
                return
            self._pending_form = dict(msg)
        self._wake.set()

    def try_enqueue(self, model: str, qnum, plan) -> bool:
        """Coordinator: queue a query as one collective round if the group covers
        its plan (one chunk per member at most)."""
        with self.lock:
            if not self.healthy:
                return False
            members = list(self.members)
        workers = [w for w, _, _ in plan]
        if len(set(workers)) != len(workers) or not set(workers) <= set(members):
            return False
        if any(e - s + 1 > self.cfg.max_chunk for _, s, e in plan):
            return False
        mid = MODEL_IDS.get(model)
        if mid is None:
            return False
        by = {w: (s, e) for w, s, e in plan}
        table = [(mid, int(qnum), by[m][0], by[m][1]) if m in by else (mid, int(qnum), 0, NO_WORK)
                 for m in members]
        self.q.put((model, qnum, table, members))
        self._wake.set()
        return True

    # -- liveness checks (polled while a collective is pending) ---------------------------
    def _check_coordinator(self, members: list[str]):
        n = self.node
        alive = set(n.membership.alive())

        def check():
            if not n.alive_flag:
                raise RoundAbandoned("node stopping")
            if not n.is_coordinator:
                raise RoundAbandoned("no longer coordinator")
            dead = [m for m in members if m not in alive and not n.membership.is_alive(m)]
            if dead:
                raise RoundAbandoned(f"member(s) {dead} failed")
        return check

    def _check_member(self, coordinator: str):
        n = self.node

        def check():
            if not n.alive_flag:
                raise RoundAbandoned("node stopping")
            if self._pending_form is not None:
                raise RoundAbandoned("newer epoch announced")
            if coordinator != n.name and not n.membership.is_alive(coordinator):
                raise RoundAbandoned(f"coordinator {coordinator} failed")
        return check

    # -- driver thread ---------------------------------------------------------------------
    def _run_chunk(self, model: str, s: int, e: int, packed=None):
        """This member's chunk of a round.  On a GPU executor the packed top-1
        pairs go straight into ``packed`` (the gather's send buffer) and None
        is returned; otherwise (cls, prob) host arrays."""
        n = self.node
        delay = self.cfg.worker_start_delay_s + n.extra_delay_s
        if delay:
            time.sleep(delay)
        t0 = time.perf_counter()
        tags = dict(model=model, start=s, end=e, epoch=self.group.epoch)
        with n.tracer.span("round.stage", **tags):
            imgs = n.source.get(s, e) if n.source is not None else None
        with n.tracer.span("round.compute", **tags):
            run_packed = getattr(n.executor, "run_packed", None)
            if run_packed is not None and packed is not None and imgs is not None and \
                    imgs.device.type == "cuda" and packed.device == imgs.device:
                run_packed(model, imgs, packed[:e - s + 1])
                out = None
            else:
                cls, prob = n.executor.run(model, imgs, s, e)
                out = np.ascontiguousarray(cls, np.int32), np.ascontiguousarray(prob, np.float32)
        n.chunks_done += 1
        self._last_compute = time.perf_counter() - t0
        return out

    def _driver(self) -> None:
        n = self.node
        while n.alive_flag:
            self._wake.wait(0.1)
            self._wake.clear()
            if not n.alive_flag:
                break
            try:
                if n.is_coordinator:
                    self._coordinator_step()
                else:
                    self._member_step()
            except Exception:  # noqa: BLE001
                log.exception("%s: round driver error", n.name)
                self._drop_group()
        self._drop_group()

    def _drop_group(self, abandoned: bool = False) -> None:
        with self.lock:
            self.healthy = False
        if abandoned:
            self.group.abort_async()          # collectives may still be pending on dead peers
        else:
            self.group.teardown()

    # coordinator -------------------------------------------------------------------------
    def _coordinator_step(self) -> None:
        n = self.node
        with self.lock:
            due = self._reform_at is not None and time.monotonic() >= self._reform_at and not self._released
            if due:
                self._reform_at = None
        if due:
            self._reform()
            return
        if self._reform_at is not None:
            self._wake.set()                       # keep polling until it is due
        if not self.group.formed:
            self._flush_queue_to_tcp()
            return
        while n.alive_flag and self._reform_at is None:
            try:
                item = self.q.get(timeout=0.05)
            except queue.Empty:
                return
            if item[0] == "__release__":
                self._stop_epoch()
                item[1].set()
                return
            model, qnum, table, members = item
            if members != self.group.members:
                self._fallback(model, qnum, table, members)
                continue
            t0 = time.perf_counter()
            try:
                out = self.group.round(table, self._run_chunk, check=self._check_coordinator(members))
            except Exception as e:  # noqa: BLE001
                self.rounds_failed += 1
                log.warning("%s: round failed in epoch %d (%s); falling back to TCP", n.name, self.group.epoch, e)
                n.tracer.instant("round.failed", epoch=self.group.epoch, q=qnum)
                self._drop_group(abandoned=True)
                self._fallback(model, qnum, table, members)
                self._flush_queue_to_tcp()
                # the failure detector re-forms on a death; re-form anyway in case it was
                # transient -- after the detector had time to drop a dead member
                self.schedule_reform("round failure", delay=self.cfg.failure_timeout_s * 1.2)
                return
            round_s = time.perf_counter() - t0
            self.rounds_done += 1
            now = time.time()
            for row, cls, prob in out:
                w = members[table.index(row)]
                # the members run in parallel: the round's wall time is each chunk's
                # (stage + compute) time as the fair-time scheduler measures it
                res = {"t": Type.RESULT, "model": model, "qnum": qnum, "start": row[2], "end": row[3],
                       "worker": w, "cls": cls.tobytes(), "prob": prob.tobytes(), "compute_s": round_s,
                       "epoch": n.membership.epoch, "t_done": now}
                n._ingest_result(dict(res, src=n.name))
                if n.standby != n.name and n.membership.is_alive(n.standby):
                    n.transport.send(n.standby, res)

    def _stop_epoch(self) -> None:
        """Let members leave the current epoch cleanly (STOP round), then drop it."""
        abandoned = False
        if self.group.formed:
            try:
                self.group.round([(0, 0, STOP, NO_WORK)] * len(self.group.members), self._run_chunk,
                                 check=self._check_coordinator(self.group.members))
            except Exception:  # noqa: BLE001
                abandoned = True
        self._drop_group(abandoned=abandoned)

    def _reform(self) -> None:
        n = self.node
        self._stop_epoch()
        self._flush_queue_to_tcp()
        members = [n.name] + [m for m in n.membership.alive() if m != n.name]
        with self.lock:
            self.epoch = max(self.epoch + 1, n.membership.epoch * 1000 + 1)
            epoch = self.epoch
            self.members = members
        if len(members) < 2:
            return                                 # nothing to collect from; TCP path only
        port = self.cfg.base_port + self.cfg.collective_port_offset + epoch % 100
        log.warning("%s: forming collective epoch %d over %s", n.name, epoch, members)
        n.tracer.instant("round.form", epoch=epoch, members=len(members))
        for m in members[1:]:
            n.transport.send(m, {"t": Type.GROUP_FORM, "epoch": epoch, "members": members, "port": port})
        ok = self.group.form(n.name, members, epoch, self.cfg.host, port)
        with self.lock:
            self.healthy = ok and self._reform_at is None and epoch == self.epoch
        if not ok:
            log.warning("%s: epoch %d rendezvous failed; TCP path until the next re-form", n.name, epoch)
            self.schedule_reform("rendezvous failed", delay=self.cfg.failure_timeout_s * 1.5)

    def _flush_queue_to_tcp(self) -> None:
        while True:
            try:
                item = self.q.get_nowait()
            except queue.Empty:
                return
            if item[0] == "__release__":
                self._stop_epoch()
                item[1].set()
                continue
            model, qnum, table, members = item
            self._fallback(model, qnum, table, members)

    def _fallback(self, model, qnum, table, members) -> None:
        """Re-send a round's chunks as TCP JOBs.  Chunks of dead members are
        re-dispatched by the failure handler (it owns the reassignment)."""
        n = self.node
        alive = set(n.membership.alive())
        for m, row in zip(members, table):
            if row[3] != NO_WORK and m in alive:
                n._send_job(m, model, qnum, row[2], row[3])

    # member ---------------------------------------------------------------------------------
    def _member_step(self) -> None:
        n = self.node
        with self.lock:
            msg, self._pending_form = self._pending_form, None
        if msg is None:
            return
        epoch, members, port = int(msg["epoch"]), list(msg["members"]), int(msg["port"])
        with self.lock:
            if epoch < self.epoch:
                return
            self.epoch, self.members = epoch, members
        if not self.group.form(n.name, members, epoch, self.cfg.host, port):
            return
        check = self._check_member(members[0])
        abandoned = False
        while n.alive_flag:
            try:
                r = self.group.round(None, self._run_chunk, check=check)
            except Exception as e:  # noqa: BLE001
                log.info("%s: left epoch %d (%s)", n.name, epoch, e)
                abandoned = True
                break
            if r == "stop":
                break
            self.rounds_done += 1
        self._drop_group(abandoned=abandoned)
        if self._pending_form is not None:
            self._wake.set()
