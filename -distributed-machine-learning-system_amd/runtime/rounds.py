"""Collective query rounds inside the fault-tolerant node runtime.

When ``cfg.collective_rounds`` is on (one node per process and per GPU, e.g.
via ``idunno.launch``), queries whose plan puts at most one chunk on each
group member run as *rounds* on the ``ElasticGroup`` instead of per-chunk TCP
JOB/RESULT messages (the reference sends every chunk and every RESULT as a TCP
message, mp4_machinelearning.py:560-613, 796-806).

One round:
  1. the coordinator sends each member its descriptor row ``(model_id, qnum,
     start, end)`` or ``None`` as a small ROUND message on the TCP control
     plane (SURVEY.md M9 "control: a per-rank work descriptor");
  2. every member stages its images, launches the HIP forward, which writes
     packed (class, prob) pairs straight into the round's device send buffer,
     and posts the gather without waiting for the GPU;
  3. ONE collective gathers the round to the coordinator (RCCL over xGMI /
     gloo), which copies it to the host once and ingests every chunk.

Space sharing.  The round table is *packed*: queued
queries whose worker sets are disjoint go into the same round, oldest first,
and a query that does not fit reserves its workers so a younger query cannot
starve it.  The scheduler gives concurrent jobs disjoint, fair-time-sized
worker subsets (``scheduler.partition``), so an AlexNet job and a ResNet18
job share every round -- on 8 GPUs they run side by side, as the reference's
jobs do on disjoint VM subsets (report Fig 2), not in turns.

Pipelining.  Send/gather/host buffers are double-buffered: the coordinator
keeps ``round_depth`` (2) rounds in flight, so a member's GPU runs round k+1
while round k is gathered and ingested, and members stage round k+1's images
while round k computes.  A member's forward does not block its host thread;
only the coordinator waits, for the oldest round's gather.

Scheduler feedback.  Each member writes the measured GPU time of one of its
earlier chunks (CUDA events around the forward) into two header rows of its
send buffer; the coordinator feeds those to the fair-time EMA, so averages
are each model's own compute time, not the round's wall time.

Liveness.  Every wait polls against the failure detector: the
coordinator abandons the in-flight rounds as soon as membership marks ANY
member dead (not only members already dead when the round began), re-sends
their chunks as TCP JOBs (results are idempotent by chunk key), aborts the
epoch's backend in the background and re-forms over the survivors.  A member
abandons when a newer epoch is announced or the coordinator is dead.  Idle
members wait for the next ROUND message on the control plane with no
collective posted, so no RCCL kernel spins on an idle GPU.
"""
from __future__ import annotations

import gc
import logging
import os
import threading
import time
from collections import deque

import numpy as np
import torch

from ..parallel.elastic import HDR_ROWS, MODEL_IDS, MODEL_NAMES, ElasticGroup, RoundAbandoned, pack_into
from .messages import Type
from .scheduler import split_range

log = logging.getLogger("idunno.rounds")


class _Query:
    __slots__ = ("model", "qnum", "rows", "members")

    def __init__(self, model, qnum, rows, members):
        self.model, self.qnum, self.rows, self.members = model, qnum, rows, members


class _Round:
    __slots__ = ("seq", "queries", "table", "work")

    def __init__(self, seq, queries, table):
        self.seq, self.queries, self.table, self.work = seq, queries, table, None


class RoundPlane:
    HDR_RING = 4        # pinned header buffers (> depth: a slot is rewritten only after its gather)
    CHECK_PERIOD_S = 0.002   # liveness re-check period inside a coordinator's poll loops
    ANNOUNCE_ROUNDS = 4      # rounds whose descriptors share one multicast frame (backlog only)
    GC_FREEZE_ROUNDS = 256   # coordinator: gc.freeze() every this many ingested rounds

    def __init__(self, node, device):
        self.node = node
        self.cfg = cfg = node.cfg
        self.group = ElasticGroup(device, backend=cfg.collective_backend or None,
                                  timeout_s=cfg.collective_timeout_s, max_chunk=cfg.max_chunk,
                                  op_timeout_s=cfg.collective_op_timeout_s, abort_join_s=cfg.abort_join_s,
                                  depth=cfg.round_depth)
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)
        self._queue: deque = deque()          # coordinator: queued _Query, FIFO
        self._round_msgs: dict = {}           # member: (epoch, seq) -> ROUND message
        self.epoch = 0                        # last epoch formed or announced
        self.members: list[str] = []
        self.healthy = False                  # coordinator: rounds may be queued
        self.rounds_done = 0
        self.rounds_failed = 0
        self.mixed_rounds = 0                 # rounds that carried more than one model
        self.mixed_splits: dict = {}          # "alexnet:3,resnet18:5" -> rounds with that worker split
        # the last mixed rounds: (seq, split key, the scheduler's averages and exact shares
        # at posting time) -- whether the split the round ran follows its own averages
        self.mixed_log: deque = deque(maxlen=128)
        self.max_queries_per_round = 0
        self.parked = True                    # member: waiting on the control plane, nothing posted
        self._inflight: deque = deque()       # this node's posted, unfinished gathers
        self._reform_at: float | None = None
        self._pending_form: dict | None = None
        self._released = False
        self._release_done = threading.Event()
        self._wake = threading.Event()
        self._thread: threading.Thread | None = None
        self._timings: deque = deque(maxlen=64)   # (model_id, n, (ev0, ev1) | seconds, cold)
        self._hdr = None
        self._tag = 0
        self._next_seq = 0                    # coordinator: seq of the next round of this epoch
        self._mirror_q = None                 # coordinator: rounds waiting for the standby mirror thread
        # coordinator host time: building / posting rounds and ingesting them (host_s), and
        # blocked on a gather (host_wait_s); bench.py reports host_s per round
        self._built_for = None                # member set of the last _build (stale sweep on change)
        self._announced: deque = deque()      # coordinator: rounds multicast but not yet posted
        self.announce_frames = 0              # descriptor frames sent (<= rounds posted)
        self.standby_rounds = 0               # standby: rounds ingested from its own gather copy
        self.host_s = 0.0
        self.host_cpu_s = 0.0                 # the same spans in driver-thread CPU time (no preemption)
        self.host_wait_s = 0.0
        self.launch_cpu_s = 0.0               # thread CPU time of this node's chunk launches
        self.host_post_s = 0.0                # of host_s: posting (descriptors, own chunk, gather)
        self.host_send_s = 0.0                # of host_post_s: ROUND descriptor sends
        self.host_release_s = 0.0             # of host_s: waiting for the standby's gather of an ingested round

    # -- lifecycle -------------------------------------------------------------------
    def start(self) -> None:
        self._thread = threading.Thread(target=self._driver, name=f"{self.node.name}-rounds", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._wake.set()
        with self.cv:
            self.cv.notify_all()
        if self._mirror_q is not None:
            self._mirror_q.put(None)              # the standby mirror thread exits

    def join(self, timeout: float = 5.0) -> None:
        """Wait for the driver thread and (bounded) for background epoch aborts
        (a process must not exit while a communicator is being torn down)."""
        th = self._thread
        if th is not None and th is not threading.current_thread():
            th.join(timeout)
        self.group.join_aborters()

    def release(self, timeout: float = 10.0) -> bool:
        """Coordinator: finish the queued rounds, end the epoch cleanly (STOP)
        and form no new one.  Used before a planned shutdown of the cluster."""
        with self.cv:
            self._released = True
            self.cv.notify_all()
        self._wake.set()
        return self._release_done.wait(timeout)

    # -- triggers (any thread) ----------------------------------------------------------
    def schedule_reform(self, reason: str, delay: float = 0.2) -> None:
        """Coordinator: re-form the group over the live members after ``delay``
        (several triggers inside the window collapse into one re-form)."""
        with self.cv:
            self.healthy = False
            at = time.monotonic() + delay
            self._reform_at = at if self._reform_at is None else min(self._reform_at, at)
            self.cv.notify_all()
        log.info("%s: re-form scheduled (%s)", self.node.name, reason)
        self._wake.set()

    def on_group_form(self, msg: dict) -> None:
        with self.cv:
            if int(msg["epoch"]) <= self.epoch:
                return
            self._pending_form = dict(msg)
            self.cv.notify_all()
        self._wake.set()

    def on_round(self, msg: dict) -> None:
        """Member: a ROUND descriptor (or STOP, or a batch of consecutive
        rounds' descriptors) from the coordinator."""
        with self.cv:
            ep = int(msg["epoch"])
            if ep < self.epoch:
                return
            batch = msg.get("batch")
            if batch is not None:
                for seq, rows in batch:
                    self._round_msgs[(ep, int(seq))] = {"t": msg["t"], "epoch": ep, "seq": int(seq), "rows": rows}
            else:
                self._round_msgs[(ep, int(msg["seq"]))] = msg
            self.cv.notify_all()
            me = self.members.index(self.node.name) if ep == self.epoch and self.node.name in self.members else -1
        if me >= 0:
            # the images of this member's announced chunks start staging now (SDFS
            # readahead in request order), not when the round loop reaches them
            for rows in ([r for _, r in batch] if batch is not None else [msg.get("rows")]):
                if rows is not None and me < len(rows) and rows[me] is not None:
                    self._readahead(rows[me][2], rows[me][3])

    def _readahead(self, s: int, e: int) -> None:
        pre = getattr(self.node.source, "prefetch", None)
        if pre is not None:
            try:
                pre(int(s), int(e))
            except Exception:  # noqa: BLE001  (best effort: the round's own get() fetches)
                log.debug("%s: readahead of [%s, %s] failed", self.node.name, s, e, exc_info=True)

    def try_enqueue(self, model: str, qnum, plan) -> bool:
        """Coordinator: queue a query for the round path if the group covers its
        plan (one chunk per member at most)."""
        with self.cv:
            if not self.healthy or self._released:
                return False
            members = tuple(self.members)
        workers = [w for w, _, _ in plan]
        if not workers or len(set(workers)) != len(workers) or not set(workers) <= set(members):
            return False
        if any(e - s + 1 > self.cfg.max_chunk for _, s, e in plan):
            return False
        if model not in MODEL_IDS:
            return False
        q = _Query(model, qnum, {w: (int(s), int(e)) for w, s, e in plan}, members)
        with self.cv:
            self._queue.append(q)
            self.cv.notify_all()
        self._wake.set()
        own = q.rows.get(self.node.name)
        if own is not None:
            self._readahead(*own)
        return True

    def stats(self) -> dict:
        g = self.group
        return {"ok": True, "epoch": g.epoch, "formed": g.formed, "members": list(g.members),
                "rounds_done": self.rounds_done, "rounds_failed": self.rounds_failed,
                "mixed_rounds": self.mixed_rounds, "mixed_splits": dict(self.mixed_splits),
                "mixed_log": list(self.mixed_log),
                "max_queries_per_round": self.max_queries_per_round,
                "parked": self.parked, "pending_collectives": self.pending_collectives(),
                "host_s": self.host_s, "host_cpu_s": self.host_cpu_s, "host_wait_s": self.host_wait_s, "host_post_s": self.host_post_s,
                "host_send_s": self.host_send_s, "host_release_s": self.host_release_s, "announce_frames": self.announce_frames, "standby_rounds": self.standby_rounds, "launch_cpu_s": self.launch_cpu_s,
                "queued": len(self._queue)}

    def collectives_quiet(self, need: bool = False) -> bool:
        """May HipExecutor's empty_cache run now?  It frees with hipFree, which
        waits for every kernel of this process on the device with the
        interpreter lock held -- a gather stuck on a peer that just died
        included, and then nothing in the process runs (heartbeats, the failure
        detector, the abort that would end the gather) until the RCCL watchdog
        fires (8-rank rehearsal, worker failover: 120 s).  True when no collective
        of this node can be pending: no epoch of more than one member formed and
        no aborted communicator still tearing down; with ``need`` (the cache
        holds more than its slack: node processes sharing one GPU) also on the
        round driver thread -- the only thread that posts collectives -- once
        every gather it posted has completed."""
        g = self.group
        if g.aborting():
            return False
        if not g.formed or len(g.members) <= 1:
            return True
        return need and threading.current_thread() is self._thread and self.pending_collectives() == 0

    def _maybe_trim(self) -> None:
        """A trim the executor had to defer (``collectives_quiet``), retried at
        the round driver's quiet points."""
        fn = getattr(self.node.executor, "maybe_trim", None)
        if fn is not None:
            fn()

    def pending_collectives(self) -> int:
        """Posted gathers of this node that have not completed."""
        works = [x.work if isinstance(x, _Round) else x[1] for x in list(self._inflight)]
        return sum(1 for w in works if w is not None and not w.is_completed())

    # -- liveness checks (polled while a collective or a descriptor is pending) -------------
    def _check_coordinator(self, members: list[str]):
        n = self.node

        others = [m for m in members if m != n.name]
        last = [0.0]

        def check():
            if not n.alive_flag:
                raise RoundAbandoned("node stopping")
            if not n.is_coordinator:
                raise RoundAbandoned("no longer coordinator")
            # the detector's verdicts move on a heartbeat period (>= 0.1 s): a poll
            # loop re-reads the member table at most every CHECK_PERIOD_S, not per spin
            t = time.perf_counter()
            if t - last[0] < self.CHECK_PERIOD_S:
                return
            last[0] = t
            # ANY member the detector now marks dead (a member that dies
            # during the round must count, not only one already dead at its start)
            dead = [m for m in others if not n.membership.is_alive(m)]
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

    # -- the work of one member in one round ------------------------------------------------
    def _run_chunk(self, row, seq: int) -> None:
        """Stage and launch this member's chunk of round ``seq`` into its send
        buffer.  A GPU executor returns at once (timing events are kept for a
        later header); a host executor is timed here."""
        n = self.node
        self._maybe_trim()
        mid, qnum, s, e = (int(v) for v in row)
        model = MODEL_NAMES[mid]
        delay = self.cfg.worker_start_delay_s + n.extra_delay_s
        if delay:
            time.sleep(delay)
        cnt = e - s + 1
        send = self.group.send_buffer(seq)
        tags = dict(model=model, q=qnum, start=s, end=e, epoch=self.group.epoch, seq=seq)
        with n.tracer.span("round.stage", **tags):
            imgs = n.source.get(s, e) if n.source is not None else None
        run_packed = getattr(n.executor, "run_packed", None)
        # a member's first chunk of a model and size (graph capture, kernel load) is
        # reported as cold: it never seeds the coordinator's fair-time average
        cold = (model, cnt) not in n.warm_shapes
        n.warm_shapes.add((model, cnt))
        c0 = time.thread_time()
        with n.tracer.span("round.launch", **tags):
            if run_packed is not None and imgs is not None and imgs.device.type == "cuda" and \
                    send.device == imgs.device:
                evs = run_packed(model, imgs, send[:cnt])
                if evs is not None:
                    self._timings.append((mid, cnt, evs, cold))
                    tl = n.gpu_timeline
                    if tl is not None:
                        tl.append(("fwd", evs[0], evs[1], cnt))
            else:
                t0 = time.perf_counter()
                cls, prob = n.executor.run(model, imgs, s, e)
                self._timings.append((mid, cnt, time.perf_counter() - t0, cold))
                pack_into(send, cls, prob)
        self.launch_cpu_s += time.thread_time() - c0     # this thread's CPU time in the launch (vs its wall span)
        n.chunks_done += 1

    def _write_header(self, seq: int) -> None:
        """Report one finished chunk's own compute time in round ``seq``'s
        header rows: (us, model_id), (n_images, tag); zeros if none finished."""
        us = mid = cnt = 0
        if self._timings:
            m, c, t, cold = self._timings[0]
            if isinstance(t, tuple):
                ev0, ev1 = t
                if ev1.query():
                    us, mid, cnt = int(ev0.elapsed_time(ev1) * 1000.0), m, c
                    self._timings.popleft()
            else:
                us, mid, cnt = int(t * 1e6), m, c
                self._timings.popleft()
            if cold:
                us = mid = cnt = 0             # measured, but not reported (see _run_chunk)
        self._tag += 1
        vals = (us, mid, cnt, self._tag)
        hdr = self.group.header(seq)
        if hdr.device.type == "cuda":
            if self._hdr is None:
                self._hdr = [torch.zeros(HDR_ROWS, 2, dtype=torch.int32, pin_memory=True)
                             for _ in range(self.HDR_RING)]
            p = self._hdr[seq % self.HDR_RING]
            p.numpy().reshape(-1)[:] = vals
            hdr.copy_(p, non_blocking=True)
        else:
            hdr.numpy().reshape(-1)[:] = vals

    # -- driver thread ---------------------------------------------------------------------
    def _driver(self) -> None:
        """Round driver thread.  IDUNNO_PROFILE_DRIVER=<path>: the coordinator's
        driver thread runs under cProfile and dumps its stats there on exit
        (host-cost diagnostics; bench.py --system)."""
        path = os.environ.get("IDUNNO_PROFILE_DRIVER")
        if not path or not self.node.is_coordinator:
            self._drive()
            return
        import cProfile

        # IDUNNO_PROFILE_DRIVER_CPU=1: the thread's CPU clock (preemption and GIL
        # waits under host contention do not count)
        pr = cProfile.Profile(time.thread_time) if os.environ.get("IDUNNO_PROFILE_DRIVER_CPU") else cProfile.Profile()
        pr.enable()
        try:
            self._drive()
        finally:
            pr.disable()
            # one file per driver thread (a re-formed plane starts a new one)
            pr.dump_stats(f"{path}.{os.getpid()}.{threading.get_ident()}")

    def _drive(self) -> None:
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
                self._drop_group(abandoned=True)
        self._drop_group(abandoned=self.group.formed)

    def _drop_group(self, abandoned: bool = False) -> None:
        with self.cv:
            self.healthy = False
        self._inflight.clear()
        if abandoned:
            self.group.abort_async()          # collectives may still be pending on dead peers
        else:
            self.group.teardown()

    # coordinator -------------------------------------------------------------------------
    def _reform_due(self) -> bool:
        with self.cv:
            return self._reform_at is not None

    def _coordinator_step(self) -> None:
        with self.cv:
            due = self._reform_at is not None and time.monotonic() >= self._reform_at and not self._released
            if due:
                self._reform_at = None
            pending = self._reform_at is not None
        if due:
            self._reform()
            return
        if pending:
            self._wake.set()                       # keep polling until it is due
            time.sleep(0.01)
            return
        if not self.group.formed:
            self._flush_queue_to_tcp()
            if self._released:
                self._release_done.set()
            return
        self._serve()

    def _build(self, members: tuple):
        """Pack the next round from the queue: oldest first, every query whose
        workers are all still free joins; a query that does not fit reserves
        its workers (no starvation).  Queued queries are first re-split onto
        the current fair-time partition (``_replan``).  Returns (queries,
        stale) where stale queries were planned for another member set (-> TCP).

        The scan stops once every member is taken or reserved (nothing further
        back can join this round), so a deep backlog costs O(members) per
        round, not O(queue); the unscanned tail keeps its order.  Stale queries
        exist only after a member-set change: the first build of an epoch
        sweeps the whole queue for them."""
        with self.cv:
            rest, self._queue = self._queue, deque()
        if not rest:
            return [], []
        take, stale, keep = [], [], []
        if self._built_for != members:
            self._built_for = members
            stale = [q for q in rest if q.members != members]
            if stale:
                rest = deque(q for q in rest if q.members == members)
        part = self._replan_part(members)
        used, reserved = set(), set()
        nm = len(members)
        while rest and len(used) + len(reserved) < nm:
            q = rest.popleft()
            if q.members != members:
                stale.append(q)
                continue
            if part is not None:
                self._replan_one(q, part)
            ws = set(q.rows)
            if ws & used or ws & reserved:
                reserved |= ws - used
                keep.append(q)
            else:
                used |= ws
                take.append(q)
        rest.extendleft(reversed(keep))
        with self.cv:
            rest.extend(self._queue)               # queued while we were packing
            self._queue = rest
        return take, stale

    def _replan_part(self, members: tuple):
        """The fair-time partition queued queries move onto (``_replan_one``),
        or None while fewer than two jobs are active."""
        n = self.node
        active = n.state.active_models()
        if len(active) < 2:
            return None
        alive = set(n.membership.alive())
        return n.sched.subsets(active, [w for w in sorted(members) if w in alive])

    def _replan_one(self, q, part: dict) -> None:
        """Move a queued (not yet posted) query onto the current partition.
        A query planned while its job ran alone holds every GPU; once a second
        job is active it is re-split onto its own fair-time subset, so the two
        jobs share the very next round instead of after the first job's backlog
        drains.  The change is a replicated job-state op (the standby sees it)."""
        tgt = part.get(q.model)
        if not tgt or set(tgt) == set(q.rows):
            return
        s0 = min(s for s, _ in q.rows.values())
        e0 = max(e for _, e in q.rows.values())
        new = [(w, s, e) for w, (s, e) in zip(tgt, split_range(s0, e0, len(tgt)))]
        if any(e - s + 1 > self.cfg.max_chunk for _, s, e in new):
            return
        old = [(w, s, e) for w, (s, e) in q.rows.items()]
        if self.node.state.replan(q.model, q.qnum, old, new):
            q.rows = {w: (s, e) for w, s, e in new}

    def _serve(self) -> None:
        """Run rounds of the current epoch until the queue is drained and a
        re-form / release / role change asks to stop (coordinator).

        With a backlog, up to ``ANNOUNCE_ROUNDS`` rounds are built at once and
        their descriptor tables go to the members in ONE multicast frame (the
        per-member send is the coordinator's largest per-round cost that grows
        with the group); each is then posted when its slot frees.  A lone query
        is announced and posted at once, as before."""
        n, g = self.node, self.group
        members = tuple(g.members)
        check = self._check_coordinator(list(members))
        inflight = self._inflight
        announced: deque = deque()              # multicast, not yet posted (members expect them)
        self._announced = announced
        idle_since = time.monotonic()
        try:
            while n.alive_flag and n.is_coordinator and not self._reform_due():
                # at most depth-1 rounds in flight when the next is posted: a slot (and the
                # members' pinned header ring) is rewritten only after its gather finished
                while len(inflight) >= g.depth:
                    self._finalize_oldest(members, check)
                while inflight and inflight[0].work.is_completed():
                    self._finalize_oldest(members, check)
                if not announced:
                    tb, cb = time.perf_counter(), time.thread_time()
                    rounds = self._build_rounds(members)
                    if rounds:
                        # owed before the multicast: a failed announce (a member lost,
                        # worker failover) falls back on these rounds' queries too
                        announced.extend(rounds)
                        self._announce(rounds, members)
                    self.host_s += time.perf_counter() - tb
                    self.host_cpu_s += time.thread_time() - cb
                if not announced:
                    if inflight:
                        # the next query (a job's window refills on ingest) may arrive
                        # while the oldest round still computes: post it as soon as it
                        # does instead of blocking on the gather
                        self._wait_queue_or(inflight[0].work, check)
                        continue
                    if self._released:
                        break
                    self._maybe_trim()
                    with self.cv:
                        if not self._queue and not self._released and self._reform_at is None:
                            self.cv.wait(0.05)
                    if time.monotonic() - idle_since > 0.5:
                        return        # hand back to the driver loop now and then (cheap)
                    continue
                idle_since = time.monotonic()
                self._post_next(announced, members)
            # rounds already announced are owed to the members (they wait for each seq)
            while announced:
                while len(inflight) >= g.depth:
                    self._finalize_oldest(members, check)
                self._post_next(announced, members)
            while inflight:
                self._finalize_oldest(members, check)
            self._stop_epoch()
            if self._released:
                self._release_done.set()
        except Exception as e:  # noqa: BLE001
            self.rounds_failed += 1
            log.warning("%s: round failed in epoch %d (%s); falling back to TCP", n.name, g.epoch, e)
            n.tracer.instant("round.failed", epoch=g.epoch)
            lost = list(inflight) + list(announced)
            announced.clear()
            self._drop_group(abandoned=True)
            for r in lost:
                for q in r.queries:
                    self._fallback_query(q)
            self._flush_queue_to_tcp()
            if self._released:
                self._release_done.set()
                return
            # the failure detector re-forms on a death; re-form anyway in case it was
            # transient -- after the detector had time to drop a dead member
            self.schedule_reform("round failure", delay=self.cfg.failure_timeout_s * 1.2)

    def _build_rounds(self, members: tuple) -> list:
        """Up to ANNOUNCE_ROUNDS consecutive rounds from the queue (stale
        queries go to the TCP path).  Rounds after the first are committed
        ahead only when they occupy every member: a partial round stays queued,
        so a query arriving meanwhile (the other job's, two-job sharing) can
        still join it."""
        out = []
        for k in range(self.ANNOUNCE_ROUNDS):
            qs, stale = self._build(members)
            for q in stale:
                self._fallback_query(q)
            if not qs:
                break
            if k and sum(len(q.rows) for q in qs) < len(members):
                with self.cv:
                    self._queue.extendleft(reversed(qs))
                break
            out.append(_Round(self._next_seq, qs, self._table(members, qs)))
            self._next_seq += 1
        return out

    def _announce(self, rounds: list, members: tuple) -> None:
        """ONE frame with the descriptor tables of ``rounds`` (member i reads
        row i of each), encoded once and written to every member's link."""
        n, g = self.node, self.group
        ts = time.perf_counter()
        rows = lambda r: [list(row) if row else None for row in r.table]      # noqa: E731
        if len(rounds) == 1:
            msg = {"t": Type.ROUND, "epoch": g.epoch, "seq": rounds[0].seq, "rows": rows(rounds[0])}
        else:
            msg = {"t": Type.ROUND, "epoch": g.epoch, "seq": rounds[0].seq,
                   "batch": [[r.seq, rows(r)] for r in rounds]}
        lost = n.transport.multicast(members[1:], msg)
        if lost:
            raise RoundAbandoned(f"ROUND {rounds[0].seq}..{rounds[-1].seq} to {lost} not delivered")
        self.host_send_s += time.perf_counter() - ts
        self.announce_frames += 1

    def _post_next(self, announced: deque, members: tuple) -> None:
        tp, cp = time.perf_counter(), time.thread_time()
        r = announced.popleft()
        self._inflight.append(r)
        self._post(r, members)
        dt = time.perf_counter() - tp
        self.host_s += dt
        self.host_post_s += dt
        self.host_cpu_s += time.thread_time() - cp

    def _wait_queue_or(self, work, check) -> None:
        t0 = time.perf_counter()
        while not work.is_completed():
            with self.cv:
                if self._queue or self._released or self._reform_at is not None:
                    return
                self.cv.wait(0.0002 if time.perf_counter() - t0 < 0.01 else 0.002)
            check()

    @staticmethod
    def _table(members: tuple, qs: list) -> list:
        table = [None] * len(members)
        idx = {m: i for i, m in enumerate(members)}
        for q in qs:
            mid = MODEL_IDS[q.model]
            for w, (s, e) in q.rows.items():
                table[idx[w]] = (mid, int(q.qnum), s, e)
        return table

    def _post(self, r: _Round, members: tuple) -> None:
        """Run the coordinator's own chunk of announced round ``r`` and post
        its gather."""
        g = self.group
        if r.table[0] is not None:
            self._run_chunk(r.table[0], r.seq)
        self._write_header(r.seq)
        r.work = g.post_gather(r.seq)
        per = {}
        for q in r.queries:
            per[q.model] = per.get(q.model, 0) + len(q.rows)
        if len(per) > 1:
            # the round table gives each member one row, so the models' worker
            # sets in this round are disjoint by construction
            self.mixed_rounds += 1
            key = ",".join(f"{m}:{c}" for m, c in sorted(per.items()))
            self.mixed_splits[key] = self.mixed_splits.get(key, 0) + 1
            sched = self.node.sched
            avg = sched.effective_avg(per)
            tot = sum(avg.values()) or 1.0
            used = sum(per.values())
            self.mixed_log.append([r.seq, key, {m: round(v, 6) for m, v in avg.items()},
                                   {m: round(avg[m] / tot * used, 2) for m in avg}])
        self.max_queries_per_round = max(self.max_queries_per_round, len(r.queries))

    def _finalize_oldest(self, members: tuple, check) -> None:
        # popped only once ingested: a round that fails here stays in flight and
        # its queries go back to the TCP path with the others
        self._finalize(self._inflight[0], members, check)
        self._inflight.popleft()

    def _finalize(self, r: _Round, members: tuple, check) -> None:
        """Wait for round ``r``'s gather, ingest every chunk with ONE job-state
        call, feed the members' measured compute times to the scheduler, and
        hand the round to the standby mirror thread (the
        host work per round is one lock hold plus O(members) array views; the
        TCP send to the standby never runs on this thread)."""
        n, g = self.node, self.group
        t_wait = time.perf_counter()
        arr = g.collect(r.seq, r.work, check)
        t0, c0 = time.perf_counter(), time.thread_time()
        self.host_wait_s += t0 - t_wait
        mc = g.max_chunk
        now = time.time()
        recs = []
        # the whole round at once: one copy of the class and probability planes
        # (every chunk's arrays are row views of them, so the host ring slot can be
        # reused), one header read and one out-of-range test for all members
        # only the rows the round's longest chunk filled (a 400-image query over 8
        # members fills 50 of max_chunk's rows): one block copy, planes as views
        lens = [0 if row is None else row[3] - row[2] + 1 for row in r.table]
        used = max(max(lens), 1)
        blk = arr[:, :used].copy()
        cls_all = blk[:, :, 0]
        prob_all = blk[:, :, 1].view(np.float32)
        hdr = arr[:, mc:mc + HDR_ROWS, :].reshape(len(arr), 2 * HDR_ROWS).tolist()  # (us, model id, n, tag)
        bad = None
        if cls_all.min() < 0:             # rare: some row holds a range-guard mark (or stale tail)
            bad = ((cls_all < 0) & (np.arange(used) < np.array(lens)[:, None])).any(axis=1).tolist()
        # every member's reported (warm) chunk is one (size, seconds) point of its
        # model's chunk-time line; the scheduler's average is that line's full-query
        # time, which does not move with how the split cut the queries
        obs = {}
        for us, hmid, cnt, _ in hdr:
            if cnt > 0 and us > 0:
                obs.setdefault(hmid, []).append((cnt, us * 1e-6))
        for hmid, pts in obs.items():
            model = MODEL_NAMES.get(hmid)
            if model is not None:
                n.sched.observe_chunks(model, pts, self.cfg.batch_for(model))
        for i, row in enumerate(r.table):
            if row is None:
                continue
            mid, qnum, s, e = row
            cls, prob = cls_all[i, :e - s + 1], prob_all[i, :e - s + 1]
            if bad is not None and bad[i]:
                # the member's split forward left fp16's range (class -2): the chunk
                # goes to it again as a TCP JOB, whose executor path reruns it on
                # the all-f32 kernels
                log.warning("%s: chunk %s %s [%d,%d] on %s exceeded the split range; rerun in fp32",
                            n.name, MODEL_NAMES[mid], qnum, s, e, members[i])
                n._send_job(members[i], MODEL_NAMES[mid], qnum, s, e)
                continue
            recs.append((MODEL_NAMES[mid], qnum, members[i], s, e, cls, prob))
        n._ingest_round(recs, now, seq=r.seq)
        self.rounds_done += 1
        if self.rounds_done % self.GC_FREEZE_ROUNDS == 0:
            # the job-state tables grow by a few objects per chunk and hold no cycles:
            # move everything allocated so far out of the cyclic collector's reach, so
            # its periodic full passes stop re-walking the whole history (-30 % host
            # time per 8-member round, tools/hostcost_probe.py)
            gc.freeze()
        sb = g.standby_rank
        if sb > 0:
            # the standby's gather of this slot too, before reuse (deferring it to the
            # slot's next post measured the same: with depth 2 that post follows at once)
            tr = time.perf_counter()
            g.release(r.work, check)
            self.host_release_s += time.perf_counter() - tr
        gathered_by_standby = sb > 0 and members[sb] == n.standby
        if recs and not gathered_by_standby and n.standby != n.name and n.membership.is_alive(n.standby):
            self._mirror(recs, now)
        self.host_s += time.perf_counter() - t0
        self.host_cpu_s += time.thread_time() - c0

    def _mirror(self, recs: list, now: float) -> None:
        """Queue a finished round for the standby (RESULTS message built and
        sent on the mirror thread).  Results are idempotent by chunk key, and
        a mirror that falls behind only delays the standby's copy."""
        if self._mirror_q is None:
            import queue

            self._mirror_q = queue.Queue()

            def run():
                n = self.node
                while n.alive_flag:
                    item = self._mirror_q.get()
                    if item is None:
                        return
                    rs, t = item
                    # the whole round as ONE frame: a row table plus two concatenated
                    # planes (not a dict + two byte strings per chunk), ingested by the
                    # standby with one record_results call
                    msg = {"t": Type.RESULTS, "rows": [[m, q, w, s, e] for m, q, w, s, e, _, _ in rs],
                           "cls": np.concatenate([r[5] for r in rs]).astype(np.int32, copy=False).tobytes(),
                           "prob": np.concatenate([r[6] for r in rs]).astype(np.float32, copy=False).tobytes(),
                           "epoch": n.membership.epoch, "t_done": t}
                    if n.standby != n.name and n.membership.is_alive(n.standby):
                        n.transport.send(n.standby, msg)

            threading.Thread(target=run, name=f"{self.node.name}-mirror", daemon=True).start()
        self._mirror_q.put((recs, now))

    def _stop_epoch(self) -> None:
        """End an idle epoch cleanly: every member gets STOP as its next round
        (it drains its gathers and shuts its backend down), then ours."""
        if not self.group.formed:
            return
        for m in self.group.members[1:]:
            self.node.transport.send(m, {"t": Type.ROUND, "epoch": self.group.epoch, "seq": self._next_seq,
                                         "stop": True})
        self._drop_group(abandoned=False)

    def _reform(self) -> None:
        n = self.node
        self._stop_epoch()                         # idle epoch (the serve loop drained it)
        self._flush_queue_to_tcp()
        members = [n.name] + [m for m in n.membership.alive() if m != n.name]
        with self.cv:
            self.epoch = max(self.epoch + 1, n.membership.epoch * 1000 + 1)
            epoch = self.epoch
            self.members = members
        # a lone node forms a one-member group: no collective, the same pipelined
        # rounds (device-resident results, one copy per round, two in flight)
        port = self.cfg.base_port + self.cfg.collective_port_offset + epoch % 100
        log.warning("%s: forming collective epoch %d over %s", n.name, epoch, members)
        n.tracer.instant("round.form", epoch=epoch, members=len(members))
        # the standby is the rounds' second gather root (it holds every finished round
        # itself, no mirror needed); every member posts the same pair of gathers
        standby = n.standby if n.standby in members[1:] else None
        for m in members[1:]:
            n.transport.send(m, {"t": Type.GROUP_FORM, "epoch": epoch, "members": members, "port": port,
                                 "standby": standby})
        others = members[1:]
        ok = self.group.form(n.name, members, epoch, self.cfg.host, port, standby=standby,
                             check=lambda: n.alive_flag and all(n.membership.is_alive(m) for m in others))
        self._next_seq = 0
        with self.cv:
            self.healthy = ok and self._reform_at is None and epoch == self.epoch
        if not ok:
            log.warning("%s: epoch %d rendezvous failed; TCP path until the next re-form", n.name, epoch)
            self.schedule_reform("rendezvous failed", delay=self.cfg.failure_timeout_s * 1.5)

    def _flush_queue_to_tcp(self) -> None:
        with self.cv:
            qs, self._queue = list(self._queue), deque()
        for q in qs:
            self._fallback_query(q)

    def _fallback_query(self, q: _Query) -> None:
        """Re-send a query's chunks as TCP JOBs.  Chunks of dead members are
        re-dispatched by the failure handler (it owns the reassignment); a
        chunk whose result is already held is dropped by the idempotent ingest."""
        n = self.node
        alive = set(n.membership.alive())
        for w, (s, e) in q.rows.items():
            if w in alive and not n.state.images_held(q.model, q.qnum, s, e):
                n._send_job(w, q.model, q.qnum, s, e)

    # member ---------------------------------------------------------------------------------
    def _member_step(self) -> None:
        n = self.node
        with self.cv:
            msg, self._pending_form = self._pending_form, None
            if msg is None:
                return
            epoch, members, port = int(msg["epoch"]), list(msg["members"]), int(msg["port"])
            if epoch < self.epoch:
                return
            self.epoch, self.members = epoch, members
            self._round_msgs = {k: v for k, v in self._round_msgs.items() if k[0] >= epoch}
        coord = members[0]

        def alive() -> bool:       # the epoch's coordinator still alive, no newer epoch announced
            return n.alive_flag and self._pending_form is None and \
                (coord == n.name or n.membership.is_alive(coord))

        if not self.group.form(n.name, members, epoch, self.cfg.host, port, standby=msg.get("standby"),
                               check=alive):
            return
        self._follow(epoch, members)
        if self._pending_form is not None:
            self._wake.set()

    def _await_round(self, epoch: int, seq: int, check, idle=None) -> dict:
        """Member: wait on the control plane (nothing posted on the GPU) for
        the coordinator's descriptor of round ``seq``.  ``idle()`` (the
        standby's drain of finished gathers) runs between waits; while it
        reports rounds still pending the wait is short."""
        while True:
            busy = idle() if idle is not None else False
            if not busy and not self._round_msgs:
                self._maybe_trim()
            with self.cv:
                msg = self._round_msgs.pop((epoch, seq), None)
                if msg is None:
                    self.parked = True
                    self.cv.wait(0.001 if busy else 0.05)
                    msg = self._round_msgs.pop((epoch, seq), None)
                if msg is not None:
                    self.parked = False
                    return msg
            check()

    def _follow(self, epoch: int, members: list[str]) -> None:
        g = self.group
        check = self._check_member(members[0])
        inflight = self._inflight
        me = members.index(self.node.name)
        standby = g.standby_rank == me          # this member is the rounds' second gather root
        abandoned = False
        seq = 0
        try:
            while True:
                msg = self._await_round(epoch, seq, check,
                                        (lambda: self._standby_drain(members, check)) if standby else None)
                if msg.get("stop"):
                    while inflight:
                        x = inflight.popleft()
                        g.wait(x[1], check)
                        if standby:
                            self._standby_ingest(x, members, check)
                    break
                while inflight and inflight[0][0] <= seq - g.depth:
                    x = inflight.popleft()
                    g.release(x[1], check)
                    if standby:
                        self._standby_ingest(x, members, check)
                rows = msg.get("rows")
                row = rows[me] if rows is not None else msg.get("row")
                if row is not None:
                    self._run_chunk(row, seq)
                self._write_header(seq)
                inflight.append([seq, g.post_gather(seq), rows, False])
                self.rounds_done += 1
                seq += 1
        except Exception as e:  # noqa: BLE001
            log.info("%s: left epoch %d (%s)", self.node.name, epoch, e)
            abandoned = True
            if standby:
                # rounds whose gather reached this standby before the coordinator (or a
                # member) failed are kept: the promoted standby does not recompute them
                for x in list(inflight):
                    try:
                        if x[1] is not None and x[1].is_completed():
                            self._standby_ingest(x, members, None)
                    except Exception:  # noqa: BLE001
                        log.debug("standby ingest of round %s failed", x[0], exc_info=True)
        self._drop_group(abandoned=abandoned)

    def _standby_drain(self, members, check) -> bool:
        """Standby: ingest every in-flight round whose gather has completed
        (kept in flight until its slot is released).  True while some round
        is not ingested yet."""
        pending = False
        for x in self._inflight:
            if not x[3]:
                if x[1] is not None and x[1].is_completed():
                    self._standby_ingest(x, members, check)
                else:
                    pending = True
        return pending

    def _standby_ingest(self, x: list, members, check) -> None:
        """Standby: record round x = [seq, work, rows, ingested] from its own
        copy of the gathered results (rows: the coordinator's descriptor
        table).  A row that left fp16's range (class < 0) is skipped: the
        coordinator reruns it and its RESULT reaches the standby too."""
        seq, work, rows, done = x
        if done or rows is None:
            return
        arr = self.group.collect(seq, work, check)
        recs = []
        for i, row in enumerate(rows):
            if row is None:
                continue
            mid, qnum, s, e = (int(v) for v in row)
            k = e - s + 1
            cls = arr[i, :k, 0].copy()
            if cls.min() < 0:
                continue
            recs.append((MODEL_NAMES[mid], qnum, members[i], s, e, cls, arr[i, :k, 1].copy().view(np.float32)))
        self.node._ingest_round(recs, time.time(), seq=seq)
        x[3] = True                  # only once held: a collect that raised is retried by the sweep
        self.standby_rounds += 1
