"""One cluster node = one rank process (one MI355X GPU) — layers L2-L6.

Re-design of the reference's monolithic ``Server`` class
(mp4_machinelearning.py:114-1334).  Every node runs the same program; roles
come from the membership state, not from host names:

  * worker       runs JOB chunks one at a time on its executor and sends each
                 RESULT to the acting coordinator *and* the hot standby
                 (instead of broadcasting to all 10 hosts, :603-613);
  * coordinator  (the acting master) accepts INFERENCE queries, splits them
                 with the fair-time scheduler, dispatches JOBs, ingests
                 RESULTs into the job-state tables, re-dispatches the chunks of
                 failed workers (:706-760), re-replicates SDFS files (:852-874)
                 and pushes structured METADATA to the standby every second;
  * hot standby  mirrors job state; when the coordinator's PINGs stop for
                 ``failure_timeout_s`` it promotes itself (new epoch), takes
                 over scheduling, re-dispatches chunks that were running on
                 dead nodes and keeps serving queries (the reference's standby
                 only ever ran whole queries locally, :592-613);
  * client       the shell: ``inference`` submits queries to the coordinator
                 with fallback to the standby (:947-969), ``c1/c2/c4/cq/cvm``
                 query the coordinator's tables.
"""
from __future__ import annotations

import logging
import os
import queue
import re
import threading
import time
from logging.handlers import RotatingFileHandler

import numpy as np

from ..models.reference import canonical
from .jobstate import JobState
from .membership import Membership
from .messages import Type
from .ring import replica_neighbors
from .scheduler import FairTimeScheduler
from .sdfs import Sdfs
from .transport import TransportError
from ..utils.tracing import Tracer

log = logging.getLogger("idunno.node")


class Node:
    def __init__(self, cfg, name: str, transport, executor, source=None, clock=time.time):
        self.cfg = cfg
        self.name = name
        self.transport = transport
        self.executor = executor
        self.source = source
        self.clock = clock
        self.membership = Membership(name, cfg, transport, master=cfg.coordinator_name)
        self.sdfs = Sdfs(self, os.path.join(cfg.store_root, name, "sdfs"))
        self.state = JobState(batchsize=cfg.batch_size, clock=clock)
        self.sched = FairTimeScheduler(budget=cfg.worker_budget)
        self.jobs: queue.Queue = queue.Queue()
        self.extra_delay_s = 0.0                   # fault injection: slow worker
        self.standby = cfg.standby_name
        self.alive_flag = True
        self.meta_seq = -1
        self._standby_ack: tuple | None = None     # (epoch, seq) the standby has applied; None = re-sync
        self.meta_bytes = 0                        # bytes of the last METADATA push (delta size check)
        self.chunks_done = 0
        self.warm_shapes: set = set()              # (model, chunk size) this node has computed once
        self._submit_lock = threading.Lock()
        self.logger = self._make_logger()
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self.promotions = 0
        self._retries: dict = {}
        self._pf: dict = {}                         # (start, end) -> Future of staged images
        self._pf_lock = threading.Lock()
        self._pf_pool = None
        self._rerep_lock = threading.Lock()     # SDFS re-replication after a failure (own thread)
        self._rerep_pool = None
        self._rerep_pending: list = []
        self._last_chunk_done: float | None = None   # worker: completion time of the previous chunk
        self.tracer = Tracer(name)
        self._progress = threading.Condition()     # notified on every ingested result (job windows)
        self._meta_lock = threading.Lock()          # one standby push at a time
        self.device = getattr(executor, "device", None)  # GPU of this node (None = CPU)
        self.rounds = None                          # collective round plane (cfg.collective_rounds)
        self.gpu_timeline: list | None = None       # bench: ("fwd", ev0, ev1, n) per round chunk when set
        self.transport.dead_check = self._peer_dead
        self.membership.on_failure.append(self._on_node_failure)
        self.membership.on_master_failure.append(self._on_master_failure)
        self.membership.on_master_change.append(self._on_master_change)
        self.membership.on_join.append(self._on_node_join)

    # -- infra --------------------------------------------------------------------
    def _make_logger(self):
        lg = logging.getLogger(f"idunno.node.{self.name}")
        lg.setLevel(logging.DEBUG)
        self.log_path = None
        if self.cfg.log_dir:
            os.makedirs(self.cfg.log_dir, exist_ok=True)
            self.log_path = os.path.join(self.cfg.log_dir, f"{self.name}.log")
            for h in list(lg.handlers):            # a previous node of this name in-process
                if isinstance(h, RotatingFileHandler) and h.baseFilename != os.path.abspath(self.log_path):
                    lg.removeHandler(h)
                    h.close()
            if not any(isinstance(h, RotatingFileHandler) for h in lg.handlers):
                h = RotatingFileHandler(self.log_path, maxBytes=100 << 20, backupCount=1)
                h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(message)s"))
                lg.addHandler(h)
            # full DEBUG log to the node's file (reference host.log); only ERROR to the console
            lg.propagate = False
            if not any(type(h) is logging.StreamHandler for h in lg.handlers):
                sh = logging.StreamHandler()
                sh.setLevel(logging.ERROR)
                lg.addHandler(sh)
        return lg

    @property
    def is_coordinator(self) -> bool:
        return self.membership.is_master()

    def start(self, join: bool = True) -> "Node":
        if self.cfg.collective_rounds and self.rounds is None:
            import torch

            from .rounds import RoundPlane

            self.rounds = RoundPlane(self, torch.device(self.device) if self.device is not None else
                                     torch.device("cpu"))
            self.rounds.start()
            if hasattr(self.executor, "trim_ok"):
                self.executor.trim_ok = self.rounds.collectives_quiet
        self.transport.start(self.handle)
        self.membership.start()
        for fn, nm in ((self._worker_loop, "worker"), (self._metadata_loop, "meta"),
                       (self._straggler_loop, "straggler")):
            th = threading.Thread(target=fn, name=f"{self.name}-{nm}", daemon=True)
            th.start()
            self._threads.append(th)
        if join:
            self.join_with_retry()
        if self.rounds is not None and self.is_coordinator:
            # the first epoch (joins re-form it; a lone node forms a one-member group)
            self.rounds.schedule_reform("start", delay=0.3)
        if self.cfg.resume and self.is_coordinator:
            def resume():   # let the workers join first
                time.sleep(self.cfg.failure_timeout_s)
                n = self.resume_from_checkpoint()
                self.logger.warning("resumed: re-sent %d chunks", n)
            threading.Thread(target=resume, name=f"{self.name}-resume", daemon=True).start()
        self.logger.info("node %s started (master=%s)", self.name, self.membership.master)
        return self

    def join_with_retry(self, timeout: float = 15.0) -> bool:
        end = time.monotonic() + timeout
        delay = 0.05
        while not self._stop.is_set():
            if self.membership.join(timeout=2.0):
                return True
            if time.monotonic() > end:
                return False
            time.sleep(delay)
            delay = min(delay * 2, 1.0)
        return False

    def stop(self) -> None:
        self._stop.set()
        self.alive_flag = False
        self.membership.stop()
        if self.rounds is not None:
            self.rounds.stop()
            self.rounds.join(timeout=5.0)
        self.jobs.put(None)
        for pool in (self._rerep_pool, self._pf_pool):
            if pool is not None:
                pool.shutdown(wait=False, cancel_futures=True)
        self.transport.close()
        close = getattr(self.executor, "close", None)
        if close is not None:
            close()

    # -- dispatch of incoming messages ---------------------------------------------------
    def handle(self, msg: dict):
        if not self.alive_flag:
            return None
        t = msg["t"]
        if t in (Type.PING, Type.PONG, Type.JOIN, Type.LEAVE, Type.PROMOTE):
            return self.membership.handle(msg)
        if t in (Type.REPLICATE, Type.FETCH, Type.UNLINK, Type.PUT, Type.GET, Type.LS, Type.DELETE,
                 Type.GET_VERSIONS, Type.HBM_HAS, Type.FETCH_HBM):
            return self.sdfs.handle(msg)
        if t == Type.INFERENCE:
            if msg.get("job"):
                return self.submit_job(msg["model"], int(msg["start"]), int(msg["end"]))
            return self.submit_query(msg["model"], int(msg["start"]), int(msg["end"]),
                                     client=msg.get("src"))
        if t == Type.JOB:
            self.jobs.put(msg)
            return {"ok": True}
        if t == Type.RESULT:
            self._ingest_result(msg)
            return None
        if t == Type.RESULTS:                   # one finished round, mirrored to the standby
            if "rows" in msg:
                self._ingest_mirrored_round(msg)
            for r in msg.get("results", []):
                self._ingest_result(dict(r, src=msg.get("src")))
            return None
        if t == Type.ROUND:
            if self.rounds is not None:
                self.rounds.on_round(msg)
            return None
        if t == Type.METADATA:
            return self._apply_metadata(msg)
        if t == Type.STATS:
            return self._stats(msg.get("view", "c1"))
        if t == Type.GREP:
            return {"ok": True, "lines": self.local_grep(msg["pattern"])}
        if t == Type.GROUP_FORM:
            if self.rounds is not None:
                self.rounds.on_group_form(msg)
            return None
        if t == Type.KILL:
            if msg.get("mode") == "delay":
                self.extra_delay_s = float(msg.get("seconds", 1.0))
                return {"ok": True}
            threading.Thread(target=self.crash, daemon=True).start()
            return None
        return {"ok": False, "error": f"unknown message {t}"}

    # -- checkpoint / resume ------------------------------------------
    def checkpoint_path(self) -> str:
        return os.path.join(self.cfg.store_root, self.name, "checkpoint.msgpack")

    def save_checkpoint(self, path: str | None = None) -> str:
        """Atomically write the coordinator state (job tables incl. results, job
        cursors, SDFS metadata, scheduler averages) to disk."""
        import msgpack

        path = path or self.checkpoint_path()
        snap = {"epoch": self.membership.epoch, "node": self.name, "time": time.time(),
                "jobs": self.state.snapshot(include_results=True), "sdfs": self.sdfs.snapshot(),
                "avg_time": dict(self.sched.avg_time)}
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(msgpack.packb(snap, use_bin_type=True))
        os.replace(tmp, path)
        return path

    def load_checkpoint(self, path: str | None = None) -> bool:
        import msgpack

        path = path or self.checkpoint_path()
        if not os.path.exists(path):
            return False
        with open(path, "rb") as f:
            snap = msgpack.unpackb(f.read(), raw=False, strict_map_key=False)
        self.state.restore(snap["jobs"])
        self.sdfs.restore(snap["sdfs"])
        self.sched.adopt(snap.get("avg_time", {}))
        self.logger.warning("restored checkpoint %s (seq %s)", path, snap["jobs"].get("seq"))
        return True

    def resume_from_checkpoint(self, path: str | None = None) -> int:
        """Coordinator restart: reload state, re-send every unfinished chunk to a
        live worker, restart unfinished coordinator-side jobs.  Returns #chunks."""
        if not self.load_checkpoint(path):
            return 0
        alive = self.membership.alive()
        n = 0
        for model, qnum, w, s, e, _t in self.state.pending():
            nw = w if w in alive else self.pick_replacement(w, alive)
            if nw is None:
                continue
            if nw != w:
                self.state.reassign(w, nw, (model, qnum, s, e))
            self._send_job(nw, model, qnum, s, e)
            n += 1
        for jid in self.state.unfinished_jobs():
            self._start_job_runner(jid)
        return n

    def _peer_dead(self, dst: str) -> bool:
        """Failure-detector view used to abandon in-flight requests early."""
        m = self.membership
        if dst == m.master and m.master_suspected:
            return True
        with m.lock:
            e = m.members.get(dst)
        return e is not None and e[1] != "RUNNING"

    def crash(self) -> None:
        """Fault injection: stop answering everything (like a killed VM)."""
        self.logger.warning("%s crashing (fault injection)", self.name)
        self.stop()

    # -- coordinator -------------------------------------------------------------------
    def submit_query(self, model: str, start: int, end: int, client: str | None = None,
                     qnum: int | None = None) -> dict:
        if not self.is_coordinator:
            if self.name == self.standby and not self.membership.is_alive(self.membership.master):
                self._promote("query arrived while coordinator is down")
            else:
                try:
                    return self.transport.request(self.membership.master,
                                                  {"t": Type.INFERENCE, "model": model, "start": start,
                                                   "end": end}, self.cfg.rpc_timeout_s)
                except TransportError:
                    if self.name != self.standby:
                        return {"ok": False, "error": "coordinator unreachable"}
                    self._promote("coordinator unreachable on forward")
        model = canonical(model)
        if end < start:
            return {"ok": False, "error": "empty range"}
        alive = self.membership.alive()
        if qnum is None:
            qnum = self.state.new_query_number(model)
        self.sched.active_jobs = self.state.active_models() | {model}
        # this job's query boundary: the fair-time split follows the current averages.
        # On the TCP path a worker still running the other job's chunks changes hands
        # only once they are done (busy); the round path re-splits queued queries
        # before they are posted, so it hands workers over at once
        rounds_ok = self.rounds is not None and self.rounds.healthy
        with self._submit_lock:       # plan + record as one step: the next plan sees these chunks busy
            plan = self.sched.assign(model, start, end, alive, boundary=True,
                                     busy=None if rounds_ok else self.state.busy_workers())
            now = self.clock()
            self.state.assign(model, qnum, plan, now)
        self.tracer.instant("query.submit", model=model, q=qnum, start=start, end=end, workers=len(plan))
        prefetch = getattr(self.source, "prefetch", None)
        if prefetch is not None:
            # this node's own chunk starts staging (SDFS shard -> HBM, background
            # thread) at submission, not when its round comes up
            for w, s, e in plan:
                if w == self.name:
                    prefetch(s, e)
        if self.rounds is not None and self.rounds.try_enqueue(model, qnum, plan):
            self.logger.info("query %s %s [%d,%d] -> collective round %s", model, qnum, start, end, plan)
            return {"ok": True, "qnum": qnum, "plan": [list(p) for p in plan], "round": True}
        for w, s, e in plan:
            self._send_job(w, model, qnum, s, e)
        self.logger.info("query %s %s [%d,%d] -> %s", model, qnum, start, end, plan)
        return {"ok": True, "qnum": qnum, "plan": [list(p) for p in plan]}

    def submit_job(self, model: str, start: int, end: int) -> dict:
        """Coordinator-side batching (the reference's two-tier variant,
        mp4_machinelearning_work_inference_separate.py:611-640):
        the client sends one whole range, the coordinator cuts it into
        batch-size queries and schedules them, paced by client_query_interval_s."""
        if not self.is_coordinator:
            return self.transport.request(self.membership.master,
                                          {"t": Type.INFERENCE, "model": model, "start": start, "end": end,
                                           "job": True}, self.cfg.rpc_timeout_s)
        model = canonical(model)
        bs = self.cfg.batch_for(model)
        jid = self.state.add_job(model, start, end, bs)
        # replicate the job before it starts: a coordinator that dies before its
        # next periodic push would otherwise take the job with it
        if self.standby != self.name:
            self.push_metadata()
        self._start_job_runner(jid)
        return {"ok": True, "job": jid, "queries": (end - start) // bs + 1}

    def _start_job_runner(self, jid: int) -> None:
        """Submit the job's remaining batch-size queries.  The job cursor lives in
        the replicated job state, so a promoted standby resumes it (skipping a
        range the old coordinator had already dispatched)."""

        def run():
            while not self._stop.is_set() and self.is_coordinator:
                with self.state.lock:
                    job = dict(self.state.jobs[jid])
                s = job["next"]
                if s > job["end"]:
                    return
                # flow control: at most job_window of this job's queries open, so every
                # query is planned (fair-time split, worker subset) against the jobs that
                # are active NOW -- a burst would plan a whole job on one split and make
                # a second job queue behind it instead of sharing the GPUs
                qlo = job["qbase"]
                qhi = qlo + (job["end"] - job["start"]) // job["bs"]
                with self._progress:
                    while not self._stop.is_set() and self.is_coordinator and \
                            self.state.open_queries(job["model"], qlo, qhi) >= max(1, self.cfg.job_window):
                        self._progress.wait(0.05)
                e = min(s + self.cfg.batch_for(job["model"]) - 1, job["end"])
                q = self.state.job_query_number(jid, s)
                # skip a query the old coordinator already dispatched (known from the
                # replicated tables) or whose results all reached this node directly
                if not self.state.range_submitted(job["model"], s, e) and \
                        not self.state.images_held(job["model"], q, s, e):
                    self.submit_query(job["model"], s, e, qnum=q)
                self.state.advance_job(jid, e + 1)
                if self.cfg.client_query_interval_s and e < job["end"]:
                    time.sleep(self.cfg.client_query_interval_s)

        threading.Thread(target=run, name=f"{self.name}-job{jid}", daemon=True).start()

    def _send_job(self, worker: str, model: str, qnum, s: int, e: int) -> bool:
        msg = {"t": Type.JOB, "model": model, "qnum": qnum, "start": s, "end": e,
               "epoch": self.membership.epoch}
        if worker == self.name:
            msg["src"] = self.name
            self.jobs.put(msg)
            return True
        ok = self.transport.send(worker, msg)
        if not ok:
            self.logger.warning("JOB to %s failed; will re-dispatch on failure detection", worker)
        return ok

    def _ingest_result(self, msg: dict) -> None:
        if "error" in msg:
            self._chunk_error(msg)
            return
        cls = np.frombuffer(msg["cls"], dtype=np.int32)
        prob = np.frombuffer(msg["prob"], dtype=np.float32)
        new = self.state.record_result(msg["model"], msg["qnum"], msg["worker"], msg["start"], msg["end"],
                                       cls, prob)
        self.tracer.instant("result.ingest", model=msg["model"], q=msg["qnum"], start=msg["start"],
                            worker=msg["worker"], new=new)
        cs = msg.get("compute_s")
        if new and cs is not None and self.is_coordinator and not msg.get("cold"):
            # (round results carry no compute_s: the members report their own GPU
            # time in the gather header instead, see rounds.RoundPlane._finalize);
            # a worker's first chunk of a model and size (graph capture) never counts
            n = msg["end"] - msg["start"] + 1
            self.sched.observe_chunk(msg["model"], n, cs, self.cfg.batch_for(msg["model"]))
        if new:
            with self._progress:
                self._progress.notify_all()

    def _ingest_round(self, recs: list, now: float, seq: int = -1) -> int:
        """Coordinator: every chunk of one finished collective round,
        [(model, qnum, worker, s, e, cls, prob)], in one job-state call; one
        trace event and one progress notification per round.  Returns the
        number of new chunks."""
        if not recs:
            return 0
        new = self.state.record_results(recs, now)
        self.tracer.instant("round.ingest", seq=seq, chunks=len(recs), new=new)
        if new:
            with self._progress:
                self._progress.notify_all()
        return new

    def _ingest_mirrored_round(self, msg: dict) -> int:
        """Standby: a round the coordinator mirrored as one frame (rounds.py
        ``_mirror``): row table + concatenated class / probability planes."""
        cls = np.frombuffer(msg["cls"], dtype=np.int32)
        prob = np.frombuffer(msg["prob"], dtype=np.float32)
        recs, o = [], 0
        for m, q, w, s, e in msg["rows"]:
            k = e - s + 1
            recs.append((m, q, w, s, e, cls[o:o + k], prob[o:o + k]))
            o += k
        if o != cls.size or o != prob.size:
            self.logger.error("mirrored round from %s: %d rows cover %d images, planes hold %d / %d",
                              msg.get("src"), len(recs), o, cls.size, prob.size)
            return 0
        return self._ingest_round(recs, self.state.clock())

    MAX_CHUNK_RETRIES = 3

    def _chunk_error(self, msg: dict) -> None:
        """A worker reported an executor failure: retry the chunk elsewhere."""
        if not self.is_coordinator:
            return
        key = (msg["model"], msg["qnum"], int(msg["start"]), int(msg["end"]))
        n = self._retries.get(key, 0) + 1
        self._retries[key] = n
        self.logger.error("chunk %s failed on %s (%s), attempt %d", key, msg["worker"], msg["error"], n)
        if n > self.MAX_CHUNK_RETRIES:
            return
        alive = [w for w in self.membership.alive() if w != msg["worker"]] or self.membership.alive()
        w = self.pick_replacement(msg["worker"], alive + [msg["worker"]])
        if w is None:
            return
        self.state.reassign(msg["worker"], w, key)
        self._send_job(w, *key)

    def pick_replacement(self, failed: str, alive: list[str]) -> str | None:
        """Least-loaded live worker, ties broken by ring order after the failed node."""
        cands = [a for a in alive if a != failed]
        if not cands:
            return None
        # ring successors of the failed node (reference :717-721), least loaded first
        order = [n for n in replica_neighbors(failed, cands) if n != failed]
        load = {w: len(self.state.chunks_of(w)) for w in order}
        return min(order, key=lambda w: (load[w], order.index(w)))

    def _on_node_join(self, node: str) -> None:
        if self.rounds is not None and self.is_coordinator:
            self.rounds.schedule_reform(f"{node} joined")

    def _on_node_failure(self, node: str) -> None:
        if not self.is_coordinator:
            return
        if self.rounds is not None:
            self.rounds.schedule_reform(f"{node} failed")
        # chunks first: the dead node's work is re-dispatched at once; SDFS
        # re-replication (seconds of file copies for a node holding shards)
        # follows on its own thread instead of delaying the recovery
        t0 = time.monotonic()
        chunks = self.state.chunks_of(node)
        alive = self.membership.alive()
        for ch in chunks:
            model, qnum, s, e = ch
            w = self.pick_replacement(node, alive)
            if w is None:
                self.logger.error("no live worker for %s", ch)
                continue
            self.state.reassign(node, w, ch)
            self._send_job(w, model, qnum, s, e)
        self.logger.warning("failure of %s: re-dispatched %d chunks in %.3fs", node, len(chunks),
                            time.monotonic() - t0)
        with self._rerep_lock:
            if self._rerep_pool is None:
                from concurrent.futures import ThreadPoolExecutor

                self._rerep_pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"{self.name}-rerep")
            self._rerep_pending.append(self._rerep_pool.submit(self._rereplicate, node))

    def _rereplicate(self, node: str) -> int:
        t0 = time.monotonic()
        try:
            moves = self.sdfs.rereplicate(node)
        except Exception:  # noqa: BLE001
            self.logger.exception("re-replication failed")
            return 0
        self.logger.warning("failure of %s: re-replicated %d files in %.3fs", node, len(moves),
                            time.monotonic() - t0)
        return len(moves)

    def wait_rereplication(self, timeout: float | None = None) -> bool:
        """Block until every re-replication started so far has finished."""
        from concurrent.futures import wait

        with self._rerep_lock:
            futs = list(self._rerep_pending)
            self._rerep_pending = [f for f in futs if not f.done()]
        return not wait(futs, timeout=timeout).not_done

    def _straggler_loop(self) -> None:
        """Resend chunks running longer than straggler_timeout_s (A7 fixed; off by default)."""
        while not self._stop.wait(max(0.05, self.cfg.straggler_timeout_s / 4)):
            if not (self.cfg.straggler_resend and self.is_coordinator):
                continue
            now = self.clock()
            for model, qnum, w, s, e, t0 in self.state.pending():
                if now - t0 > self.cfg.straggler_timeout_s:
                    alt = self.pick_replacement(w, self.membership.alive())
                    if alt:
                        self.logger.warning("straggler %s %s [%d,%d] on %s -> %s", model, qnum, s, e, w, alt)
                        self.state.reassign(w, alt, (model, qnum, s, e))
                        self._send_job(alt, model, qnum, s, e)

    # -- standby replication ------------------------------------------------------------
    def _metadata_loop(self) -> None:
        last_ckpt = time.monotonic()
        while not self._stop.wait(self.cfg.metadata_period_s):
            if not self.is_coordinator:
                continue
            if self.standby != self.name:
                self.push_metadata()
            if self.cfg.checkpoint_period_s > 0 and time.monotonic() - last_ckpt >= self.cfg.checkpoint_period_s:
                try:
                    self.save_checkpoint()
                except OSError:
                    self.logger.exception("checkpoint failed")
                last_ckpt = time.monotonic()

    def push_metadata(self) -> bool:
        """Replicate the job state to the hot standby: the job-table mutations
        since the standby's last acknowledged sequence number (a full snapshot
        only on first contact, after a gap, or when the log was truncated),
        plus the small SDFS / scheduler tables.  Request/reply, so the ack
        drives the next push (reference: a full str() dump every second,
        mp4_machinelearning.py:971-987)."""
        import msgpack

        if not self.membership.is_alive(self.standby):
            return False                  # a dead standby must not stall submission / checkpoints
        with self._meta_lock:             # one push at a time: acks never race backwards
            return self._push_metadata(msgpack)

    def _push_metadata(self, msgpack) -> bool:
        epoch = self.membership.epoch
        ack = self._standby_ack
        deltas = None
        if ack is not None and ack[0] == epoch:
            deltas = self.state.deltas_since(ack[1])
        msg = {"t": Type.METADATA, "seq": self.state.seq, "epoch": epoch, "sdfs": self.sdfs.snapshot(),
               "avg_time": dict(self.sched.avg_time)}
        if deltas is None:
            msg.update(kind="snapshot", jobs=self.state.snapshot(include_results=False))
        else:
            msg.update(kind="delta", base=ack[1], deltas=deltas)
        self.meta_bytes = len(msgpack.packb(msg, use_bin_type=True))
        try:
            r = self.transport.request(self.standby, msg, self.cfg.rpc_timeout_s)
        except TransportError:
            return False
        if r and r.get("ok") and "seq" in r:
            self._standby_ack = (epoch, int(r["seq"]))
            return True
        self._standby_ack = None if not r or r.get("resync") else (epoch, int(r.get("seq", 0)))
        return False

    def _apply_metadata(self, msg: dict) -> dict:
        if self.is_coordinator:
            return {"ok": False, "resync": True, "error": "coordinator does not mirror"}
        epoch = int(msg.get("epoch", 0))
        if epoch < self.membership.epoch:
            return {"ok": False, "resync": True, "error": "stale epoch"}
        if msg.get("kind", "snapshot") == "snapshot":
            self.state.restore(msg["jobs"], keep_results=True)
            self._mirror_epoch = epoch
        else:
            if getattr(self, "_mirror_epoch", None) != epoch or int(msg["base"]) > self.state.mirror_seq:
                return {"ok": False, "resync": True, "seq": self.state.mirror_seq}
            if not self.state.apply_deltas(msg["deltas"]):
                return {"ok": False, "resync": True, "seq": self.state.mirror_seq}
        self.sdfs.restore(msg["sdfs"])
        self.sched.adopt(msg.get("avg_time", {}))
        self.meta_seq = self.state.mirror_seq
        return {"ok": True, "seq": self.state.mirror_seq}

    def _on_master_failure(self, old: str) -> None:
        if self.name == self.standby:
            self._promote(f"no heartbeat from {old}")

    def _promote(self, why: str) -> None:
        if self.is_coordinator:
            return
        old = self.membership.master
        epoch = self.membership.epoch + 1
        t0 = time.monotonic()
        self.logger.warning("%s promoting to coordinator (epoch %d): %s", self.name, epoch, why)
        self.membership.become_master(epoch)
        self.promotions += 1
        self._standby_ack = None
        for n in self.membership.alive():
            if n not in (self.name, old):
                self.transport.send(n, {"t": Type.PROMOTE, "epoch": epoch})
        # the old coordinator is gone: its own chunks and replicas must move
        self.membership.mark_failed(old)
        reopened = self.state.reopen_unheld()
        if reopened:
            self.logger.warning("%d chunk(s) finished only at %s: recomputing", reopened, old)
        # Every chunk still pending in the replicated tables is (re)sent: to a
        # replacement if its worker is dead, else to the same worker again.  A
        # chunk the old coordinator recorded (and replicated) but crashed before
        # sending would otherwise stay pending forever; for one that is already
        # in flight the duplicate answer is dropped by the idempotent ingest.
        alive = set(self.membership.alive())
        for model, qnum, w, s, e, _t in self.state.pending():
            if w not in alive:
                nw = self.pick_replacement(w, sorted(alive))
                if nw:
                    self.state.reassign(w, nw, (model, qnum, s, e))
                    self._send_job(nw, model, qnum, s, e)
            else:
                self._send_job(w, model, qnum, s, e)
        for jid in self.state.unfinished_jobs():      # coordinator-side jobs carry on here
            self._start_job_runner(jid)
        self.logger.warning("promotion done in %.3fs", time.monotonic() - t0)

    def _on_master_change(self, new: str, epoch: int) -> None:
        self.logger.info("master is now %s (epoch %d)", new, epoch)
        if self.rounds is not None and new == self.name:
            self.rounds.schedule_reform(f"promoted (epoch {epoch})", delay=0.5)

    # -- worker ---------------------------------------------------------------------------
    def _prefetch_next(self) -> None:
        """Stage the images of the next queued JOB on a helper thread while the
        current chunk computes (SURVEY.md §2.7 "double-buffered staging"): the
        SDFS shard fetch + host->HBM copy of chunk k+1 overlaps the forward of
        chunk k.  At most one chunk ahead."""
        if self.source is None or not self.cfg.prefetch:
            return
        with self.jobs.mutex:
            nxt = next((m for m in self.jobs.queue if m is not None), None)
        if nxt is None:
            return
        key = (int(nxt["start"]), int(nxt["end"]))
        with self._pf_lock:
            if key in self._pf or len(self._pf) >= 2:
                return
            if self._pf_pool is None:
                from concurrent.futures import ThreadPoolExecutor

                self._pf_pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"{self.name}-prefetch")
            tags = dict(model=nxt["model"], q=nxt["qnum"], start=key[0], end=key[1], prefetch=True)

            dev = self.device

            def stage():
                import contextlib

                import torch

                ctx = torch.cuda.device(dev) if dev is not None and torch.device(dev).type == "cuda" \
                    else contextlib.nullcontext()
                with ctx, self.tracer.span("chunk.stage", **tags):
                    imgs = self.source.get(*key)
                    if imgs is not None and imgs.device.type == "cuda":
                        torch.cuda.current_stream(imgs.device).synchronize()   # staged before handing over
                    return imgs
            self._pf[key] = self._pf_pool.submit(stage)

    def _staged(self, s: int, e: int):
        """Images of [s, e]: the prefetched tensor if one is ready or in flight."""
        with self._pf_lock:
            fut = self._pf.pop((s, e), None)
        if fut is not None:
            try:
                return fut.result()
            except Exception:  # noqa: BLE001  (fall through to a direct fetch)
                self.logger.exception("prefetch of [%d,%d] failed", s, e)
        return self.source.get(s, e) if self.source is not None else None

    def _worker_loop(self) -> None:
        """JOB queue -> executor, two chunks deep: chunk k+1 is launched before
        chunk k's results are read back and sent, so the host-side result path
        (read-back, RESULT messages, ingest) overlaps the next forward."""
        pending = None
        while not self._stop.is_set():
            if pending is None:
                msg = self.jobs.get()
            else:
                try:
                    msg = self.jobs.get_nowait()
                except queue.Empty:
                    self._finish_safe(pending)
                    pending = None
                    continue
            if msg is None or self._stop.is_set():
                if pending is not None:
                    self._finish_safe(pending)
                return
            if pending is not None and not self._quick_start(msg):
                # a pause (fault-injection delay) or a slow staging (cold SDFS
                # shard) ahead: answer the finished chunk first
                self._finish_safe(pending)
                pending = None
            try:
                ctx = self.start_chunk(msg)
            except Exception as e:  # noqa: BLE001
                self._chunk_failed(msg, e)
                ctx = None
            if pending is not None:
                self._finish_safe(pending)
            pending = ctx

    def _quick_start(self, msg: dict) -> bool:
        """Whether start_chunk(msg) launches without a pause: no configured
        delay, and its images are prefetched, cached or synthesised."""
        if self.cfg.worker_start_delay_s + self.extra_delay_s > 0:
            return False
        key = (int(msg["start"]), int(msg["end"]))
        with self._pf_lock:
            fut = self._pf.get(key)
        if fut is not None:
            # the prefetch was queued a moment ago (start_chunk of the previous
            # chunk): a synthesised or cached stage completes within a few ms, so
            # give it that long before treating it as slow -- answering the
            # finished chunk first would leave the GPU idle while this one stages
            try:
                fut.result(timeout=self.cfg.quick_start_wait_s)
            except Exception:  # noqa: BLE001  (timeout, or a failed prefetch start_chunk reports)
                pass
            return fut.done()
        cached = getattr(self.source, "cached", None)
        return cached is None or cached(*key)

    def _chunk_failed(self, msg: dict, e: Exception) -> None:
        self.logger.exception("chunk failed: %s", msg)
        err = {"t": Type.RESULT, "model": msg["model"], "qnum": msg["qnum"], "start": msg["start"],
               "end": msg["end"], "worker": self.name, "error": f"{type(e).__name__}: {e}"}
        if self.membership.master == self.name:
            self._ingest_result(dict(err, src=self.name))
        else:
            self.transport.send(self.membership.master, err)

    def _finish_safe(self, ctx) -> None:
        try:
            self.finish_chunk(ctx)
        except Exception as e:  # noqa: BLE001
            self._chunk_failed(ctx[0], e)

    def run_chunk(self, msg: dict) -> None:
        self.finish_chunk(self.start_chunk(msg))

    def start_chunk(self, msg: dict):
        """Stage the chunk's images and launch its forward (returns at once on
        an asynchronous executor)."""
        delay = self.cfg.worker_start_delay_s + self.extra_delay_s
        if delay:
            time.sleep(delay)
        model, s, e = msg["model"], int(msg["start"]), int(msg["end"])
        t0 = time.perf_counter()
        tags = dict(model=model, q=msg["qnum"], start=s, end=e)
        with self.tracer.span("chunk.stage", **tags):
            imgs = self._staged(s, e)
        self._prefetch_next()                 # next JOB's images stage while this one computes
        t_launch = time.time()
        handle = self.executor.submit(model, imgs, s, e)
        # a synchronous executor ran the chunk inside submit(): its own time is that
        # call plus the staging (the pipelined worker finishes chunk k only after
        # chunk k+1 ran, so completion-to-completion would not measure it)
        sync_dt = time.perf_counter() - t0 if getattr(handle, "synchronous", False) else None
        return (msg, t0, tags, t_launch, handle, sync_dt)

    def finish_chunk(self, ctx) -> None:
        """Wait for a launched chunk, send / ingest its RESULT."""
        msg, t0, tags, t_launch, handle, sync_dt = ctx
        cls, prob = handle.result()
        t_done = time.time()
        self.tracer.complete("chunk.compute", t_launch, t_done, **tags)
        # its own time: from launch, or from the previous chunk's completion if
        # it had to queue behind that one on the GPU (fair-time averages)
        prev = self._last_chunk_done
        self._last_chunk_done = t_done
        dt = sync_dt if sync_dt is not None else \
            (time.perf_counter() - t0) if prev is None or prev <= t_launch else (t_done - prev)
        if not self.alive_flag:
            return
        model, s, e = msg["model"], int(msg["start"]), int(msg["end"])
        shape = (model, e - s + 1)
        cold = shape not in self.warm_shapes
        self.warm_shapes.add(shape)
        res = {"t": Type.RESULT, "model": model, "qnum": msg["qnum"], "start": s, "end": e,
               "worker": self.name, "cls": np.ascontiguousarray(cls, np.int32).tobytes(),
               "prob": np.ascontiguousarray(prob, np.float32).tobytes(), "compute_s": dt,
               "epoch": msg.get("epoch", 0)}
        if cold:
            res["cold"] = True
        self.chunks_done += 1
        targets = {self.membership.master, self.standby}
        for dst in targets:
            if dst == self.name:
                self._ingest_result(dict(res, src=self.name))
            else:
                self.transport.send(dst, dict(res))

    # -- views -----------------------------------------------------------------------------
    def _stats(self, view: str) -> dict:
        v = view.lower()
        if v == "c1":
            return {"ok": True, "text": self.state.c1()}
        if v == "c2":
            return {"ok": True, "text": self.state.c2()}
        if v == "c4":
            return {"ok": True, "results": self.state.inference_result_list()}
        if v == "cq":
            return {"ok": True, "text": self.state.cq()}
        if v in ("cvm", "c5"):
            return {"ok": True, "text": self.state.cvm()}
        if v == "trace":
            return {"ok": True, "events": self.tracer.export()}
        if v == "checkpoint":
            return {"ok": True, "path": self.save_checkpoint()}
        if v == "summary":
            return self.state.summary()
        if v == "rounds":
            return self.rounds.stats() if self.rounds is not None else {"ok": False, "error": "no rounds"}
        if v == "sched":
            return {"ok": True, "avg_time": dict(self.sched.avg_time)}
        return {"ok": False, "error": f"unknown view {view}"}

    def local_grep(self, pattern: str) -> list[str]:
        """MP1 distributed-grep replacement: regex over this node's log."""
        if not self.log_path or not os.path.exists(self.log_path):
            return []
        rx = re.compile(pattern)
        with open(self.log_path, errors="replace") as f:
            return [f"{self.name}: {ln.rstrip()}" for ln in f if rx.search(ln)]
