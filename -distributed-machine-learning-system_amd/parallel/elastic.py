"""Epoch-versioned collective group for the fault-tolerant node runtime
(SURVEY.md §5.8 "RCCL fault tolerance", §7.3 hard part 2).

The steady-state query path of a healthy cluster runs in *rounds* (see
``idunno.runtime.rounds``): the coordinator sends every member its work
descriptor over the TCP control plane (SURVEY.md M9 "control: a per-rank work
descriptor"), each member writes its packed top-1 pairs into a device send
buffer, and ONE collective gathers them to the coordinator (M11, RCCL over
xGMI on MI355X, gloo on CPU).  The reference has no collective at all (every
RESULT is a TCP message to all 10 hosts, mp4_machinelearning.py:603-613).

Design points:

  * **No default process group.**  Each epoch is its own backend object
    (``ProcessGroupNCCL`` / ``ProcessGroupGloo``) built on a ``PrefixStore``
    of a TCPStore hosted by the coordinator.  An old epoch can still be
    aborting on a background thread while the next one forms, so a stuck
    ``ncclCommAbort`` never delays the re-form, and no
    private ``torch.distributed`` API is needed: ``Backend.abort()`` /
    ``shutdown()`` are public, and the process-group timeout is given at
    construction.
  * **Double-buffered rounds.**  Send, gather and host buffers come in
    ``depth`` slots (round ``seq`` uses slot ``seq % depth``) so round k+1
    computes while round k's gather and ingest run.
  * **Results stay on the device until one copy.**  A member's forward writes
    (class, prob bits) straight into ``send_buffer(seq)``; the coordinator
    copies the whole gathered round to pinned host memory once, on a side
    stream that does not wait for the compute queued behind it.
  * **Liveness from the failure detector.**  Every wait polls ``work`` in
    short slices against a caller check (membership of the members, a newer
    epoch, node shutdown) that raises ``RoundAbandoned``; the process-group
    timeout (``op_timeout_s``) is only a backstop.  Members idle between
    queries wait on the TCP control plane, never inside a posted collective.

Each send buffer ends with ``HDR_ROWS`` header rows the member fills with the
measured compute time of one of its earlier chunks (``(us, model_id),
(n_images, tag)``), so the coordinator's fair-time scheduler learns each
model's own compute time rather than the round's wall time.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from datetime import timedelta

import numpy as np
import torch
import torch.distributed as dist

log = logging.getLogger("idunno.elastic")

MODEL_IDS = {"alexnet": 0, "resnet18": 1, "resnet50": 2, "resnet34": 3}
MODEL_NAMES = {v: k for k, v in MODEL_IDS.items()}
HDR_ROWS = 2        # (compute_us, model_id), (n_images, tag) at the end of every send buffer


class RoundAbandoned(RuntimeError):
    """A round's liveness check failed (dead rank, newer epoch, shutdown)."""


class _Solo:
    """The backend of a one-member group: nothing to talk to.  A single-GPU
    node still runs its queries as pipelined rounds (device-resident results,
    one device->host copy per round, two rounds in flight), just without a
    collective."""

    def abort(self):
        pass

    def shutdown(self):
        pass


class _PairWork:
    """Both gathers of a round (coordinator root, standby root) as one handle."""

    def __init__(self, *works):
        self.works = works

    def is_completed(self) -> bool:
        return all(w.is_completed() for w in self.works)

    def wait(self):
        for w in self.works:
            w.wait()
        return True


class _EventWork:
    """Work-like handle of a solo round: complete once the round's kernels
    (recorded event) have finished; nothing to wait for on the CPU."""

    def __init__(self, ev=None):
        self.ev = ev

    def is_completed(self) -> bool:
        return self.ev is None or self.ev.query()

    def wait(self):
        return True


def _shutdown_backend(pg, abort: bool) -> None:
    """End a backend object: ``abort()`` when collectives may still be
    pending on a dead peer (RCCL: ncclCommAbort, pending kernels return),
    else ``shutdown()`` where the backend has it."""
    fn = None
    if not abort:
        fn = getattr(pg, "shutdown", None)
    if fn is None:
        fn = getattr(pg, "abort", None)
    if fn is not None:
        fn()


class ElasticGroup:
    def __init__(self, device: torch.device, backend: str | None = None, timeout_s: float = 30.0,
                 max_chunk: int = 1024, op_timeout_s: float = 120.0, abort_join_s: float = 5.0,
                 depth: int = 2, solo: bool = True):
        self.device = torch.device(device)
        # solo: a one-member epoch runs without a backend (_Solo); False builds the
        # real one even then (the GPU test of the RCCL path on a one-GPU box)
        self.solo = solo
        self.backend = backend or ("nccl" if self.device.type == "cuda" else "gloo")
        self.timeout_s = timeout_s            # rendezvous (store + backend construction)
        self.op_timeout_s = op_timeout_s      # backstop for one collective; liveness comes from check()
        self.abort_join_s = abort_join_s      # how long teardown waits for a background abort
        self.max_chunk = max_chunk
        self.depth = depth
        self.epoch = -1
        self.members: list[str] = []
        self.rank = -1
        self.pg = None
        self.lock = threading.RLock()
        self._store = None
        self._aborters: list[threading.Thread] = []
        self.poll_s = 0.0005
        self.standby_rank = -1                # second gather root (the hot standby), -1: none
        self._send = self._gathered = self._host = None
        self._gopt: dict = {}                      # root rank -> GatherOptions
        self._d2h = None

    @property
    def formed(self) -> bool:
        return self.pg is not None

    @property
    def world(self) -> int:
        return len(self.members)

    def describe(self) -> dict:
        """The live epoch's backend as the process group reports it: name
        ("nccl" = RCCL on ROCm, "gloo"; "solo" for a one-member group) and
        size.  Empty when no epoch is formed."""
        pg = self.pg
        if pg is None:
            return {}
        if isinstance(pg, _Solo):
            return {"backend": "solo (one member, no collective)", "world": 1, "epoch": self.epoch}
        name = pg.name() if hasattr(pg, "name") else self.backend
        return {"backend": str(name).lower(), "world": int(pg.size()), "epoch": self.epoch,
                "rccl": self.backend == "nccl" and torch.version.hip is not None}

    # -- lifecycle ---------------------------------------------------------------
    def _detach(self):
        pg, self.pg = self.pg, None
        self._store = None
        self._send = self._gathered = self._host = None
        return pg

    def teardown(self) -> None:
        """Clean teardown of a healthy group (no collective in flight)."""
        with self.lock:
            pg = self._detach()
        if pg is not None:
            try:
                _shutdown_backend(pg, abort=False)
            except Exception:  # noqa: BLE001  (a broken group can fail to clean up)
                log.exception("backend shutdown failed")

    def abort_async(self) -> None:
        """Abandon the current epoch with collectives possibly still pending:
        abort its backend on a background thread so the caller never blocks
        on a dead peer.  The next epoch does not wait for it (own backend)."""
        with self.lock:
            pg = self._detach()
            if pg is None:
                return

            def run():
                try:
                    _shutdown_backend(pg, abort=True)
                except Exception:  # noqa: BLE001
                    log.exception("abort of the old epoch failed")

            th = threading.Thread(target=run, name="epoch-abort", daemon=True)
            th.start()
            self._aborters = [t for t in self._aborters if t.is_alive()] + [th]

    def aborting(self) -> bool:
        """A communicator abort is still running on a background thread (its
        collectives may still be on the device)."""
        return any(t.is_alive() for t in list(self._aborters))

    def join_aborters(self, timeout: float | None = None) -> bool:
        """Wait (bounded by ``abort_join_s``) for background aborts to end;
        True if none is left running.  Used before a process exits."""
        end = time.monotonic() + (self.abort_join_s if timeout is None else timeout)
        for th in list(self._aborters):
            th.join(max(0.0, end - time.monotonic()))
        self._aborters = [t for t in self._aborters if t.is_alive()]
        return not self._aborters

    def form(self, me: str, members: list[str], epoch: int, host: str, port: int,
             standby: str | None = None, check=None) -> bool:
        """Join epoch ``epoch`` (blocking rendezvous of all ``members``; rank 0
        = members[0] hosts the TCPStore).  With ``standby`` (a member other
        than rank 0) every round is gathered to it as well (the
        reference sends every RESULT to the standby too,
        mp4_machinelearning.py:603-613), so a promoted standby already holds
        the rounds that completed before the coordinator died.  Every member
        must be given the same ``standby``.  ``check()`` (the failure detector:
        False once a member of the epoch is dead) is polled while the RCCL
        communicator is set up: a member killed inside that set-up would
        otherwise block every other member's form() in the backend's bootstrap
        (bench --rehearse-rccl coordinator failover at N >= 4, round 5).
        Returns False on failure."""
        with self.lock:
            self.teardown()
            if me not in members:
                return False
            rank = members.index(me)
            world = len(members)
            self.standby_rank = members.index(standby) if standby in members[1:] else -1
            if world == 1 and self.solo:
                self.pg = _Solo()
                self.epoch, self.members, self.rank = epoch, list(members), 0
                self._alloc(1)
                return True
            try:
                store = dist.TCPStore(host, port, world_size=world, is_master=(rank == 0),
                                      timeout=timedelta(seconds=self.timeout_s), wait_for_workers=False,
                                      use_libuv=False)
                pstore = dist.PrefixStore(f"epoch{epoch}", store)
                op_to = timedelta(seconds=self.op_timeout_s)
                if self.backend == "nccl":
                    # on a collective timeout abort the communicator, never the process
                    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
                    torch.cuda.set_device(self.device)
                    pg = dist.ProcessGroupNCCL(pstore, rank, world, op_to)
                    # communicator set-up now, while every member is in form()
                    eager = getattr(pg, "eager_connect_single_device", None)
                    if eager is not None and not self._connect(pg, eager, check):
                        log.warning("%s: epoch %d: a member failed during communicator set-up", me, epoch)
                        return False
                else:
                    pg = dist.ProcessGroupGloo(pstore, rank, world, op_to)
            except Exception:  # noqa: BLE001
                log.exception("%s: forming epoch %d failed", me, epoch)
                return False
            self._store = store
            self.pg = pg
            self.epoch, self.members, self.rank = epoch, list(members), rank
            self._alloc(world)
            if self.backend == "nccl" and not self._warm_up(check):
                log.error("%s: epoch %d: warm-up gather did not complete", me, epoch)
                self.abort_async()
                return False
            return True

    def _connect(self, pg, eager, check) -> bool:
        """Run the blocking communicator set-up on a helper thread and poll
        ``check`` meanwhile; a failed check (or the store timeout) aborts the
        communicator from here, which ends the set-up on every live member."""
        done, err = threading.Event(), []

        def run():
            try:
                eager(self.device)
            except Exception as e:  # noqa: BLE001
                err.append(e)
            done.set()

        th = threading.Thread(target=run, name="rccl-connect", daemon=True)
        th.start()
        end = time.monotonic() + self.timeout_s
        while not done.wait(0.01):
            if (check is not None and not check()) or time.monotonic() > end:
                self._abort_in_background(pg)
                return False
        if err:
            # a set-up that raised leaves a half-built communicator: end it too
            self._abort_in_background(pg)
            return False
        return True

    def _abort_in_background(self, pg) -> None:
        def abort():
            try:
                _shutdown_backend(pg, abort=True)
            except Exception:  # noqa: BLE001
                log.exception("abort of a communicator in set-up failed")

        ab = threading.Thread(target=abort, name="rccl-abort", daemon=True)
        ab.start()
        self._aborters = [t for t in self._aborters if t.is_alive()] + [ab]

    def _warm_up(self, check=None) -> bool:
        """One gather (pair) of every member while all of them are still in
        ``form()``: RCCL sets up a pair's point-to-point connection at the pair's
        first operation, and that handshake blocks the POSTING thread until the
        peer posts too.  Without it the coordinator's first post of an epoch
        waited on a member paused in its chunk, and when that member was killed,
        for the backend's whole timeout (120 s) instead of the failure detector's
        2 s (bench --rehearse-rccl worker failover, round 5).  ``check`` (the
        failure detector, as in ``form``) is polled too: a member that dies
        between the set-up and the warm-up ends the wait at once, not after
        ``timeout_s`` (the caller aborts the epoch)."""
        work = self.post_gather(0)
        end = time.monotonic() + self.timeout_s
        while not work.is_completed():
            if time.monotonic() > end or (check is not None and not check()):
                return False
            time.sleep(0.001)
        work.wait()
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        return True

    def _alloc(self, world: int) -> None:
        dev, rows, D = self.device, self.max_chunk + HDR_ROWS, self.depth
        self._send = [torch.zeros(rows, 2, dtype=torch.int32, device=dev) for _ in range(D)]
        self._send_list = [[t] for t in self._send]          # gather input lists, built once
        root = self.rank == 0 or self.rank == self.standby_rank
        if isinstance(self.pg, _Solo):
            self._gathered = [s.unsqueeze(0) for s in self._send]       # the send buffer IS the round
        elif root:
            self._gathered = [torch.zeros(world, rows, 2, dtype=torch.int32, device=dev) for _ in range(D)]
            # per-slot gather output lists, built once (not one unbind per round)
            self._gather_outs = [[list(g.unbind(0))] for g in self._gathered]
        if root:
            gpu = dev.type == "cuda"
            self._host = [torch.zeros(world, rows, 2, dtype=torch.int32, pin_memory=gpu) for _ in range(D)]
            if gpu and self._d2h is None:
                self._d2h = torch.cuda.Stream(device=dev)

    # -- buffers -----------------------------------------------------------------
    def send_buffer(self, seq: int) -> torch.Tensor:
        """[max_chunk, 2] int32 (class, prob bits) of round ``seq``."""
        return self._send[seq % self.depth][: self.max_chunk]

    def header(self, seq: int) -> torch.Tensor:
        return self._send[seq % self.depth][self.max_chunk:]

    # -- collectives -----------------------------------------------------------------
    def post_gather(self, seq: int):
        """Start the gather of round ``seq``'s send buffer to rank 0 (Work)."""
        pg = self.pg
        if pg is None:
            raise RoundAbandoned("group not formed")
        if isinstance(pg, _Solo):
            ev = None
            if self.device.type == "cuda":
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
            return _EventWork(ev)
        slot = seq % self.depth
        outs = self._gather_outs[slot] if self.rank == 0 else []
        work = pg.gather(outs, self._send_list[slot], self._gopts(0))
        sb = self.standby_rank
        if sb <= 0:
            return work
        return _PairWork(work, pg.gather(self._gather_outs[slot] if self.rank == sb else [], self._send_list[slot],
                                         self._gopts(sb)))

    def _gopts(self, root: int):
        """GatherOptions per root, built once (two per round otherwise)."""
        o = self._gopt.get(root)
        if o is None:
            o = self._gopt[root] = dist.GatherOptions()
            o.rootRank = root
        return o

    def wait(self, work, check=None, spin_s: float = 0.001) -> None:
        """Poll ``work`` until it completes; ``check()`` raises RoundAbandoned
        (liveness) between polls.  Spins ``spin_s`` (the coordinator's gather:
        on the critical path), then sleeps ``poll_s``, backing off to 4x after
        10 ms and 20x after 1 s."""
        if work is None:
            return
        t0 = time.perf_counter()
        while not work.is_completed():
            if check is not None:
                check()
            if self.pg is None:
                raise RoundAbandoned("epoch torn down")
            waited = time.perf_counter() - t0
            if waited >= spin_s:
                time.sleep(self.poll_s * (1 if waited < 0.01 else 4 if waited < 1.0 else 20))
        work.wait()

    def release(self, work, check=None) -> None:
        """Member: the slot of a finished round may be rewritten once its
        gather is done.  On the GPU this is a stream dependency (the next
        forward on the current stream waits for the gather, the host does
        not); on the CPU the gather is polled to completion."""
        if work is None:
            return
        if self.device.type == "cuda":
            work.wait()
        else:
            # off the critical path (the slot is reused depth rounds later): sleep
            # between polls instead of spinning a core the coordinator needs
            self.wait(work, check, spin_s=0.0)

    def collect(self, seq: int, work, check=None) -> np.ndarray:
        """A gather root (rank 0, or the standby): wait for round ``seq``'s
        gather and return the whole round
        as host int32 [world, max_chunk + HDR_ROWS, 2] (one device->host copy
        on a side stream: compute queued on the current stream is not waited
        for).  Of a gather pair only this root's own gather is waited for; the
        caller releases the pair before the slot is rewritten."""
        if isinstance(work, _PairWork):
            work = work.works[0 if self.rank == 0 else 1]
        self.wait(work, check)
        slot = seq % self.depth
        host = self._host[slot]
        if self.device.type == "cuda":
            with torch.cuda.stream(self._d2h):
                host.copy_(self._gathered[slot], non_blocking=True)
            self._d2h.synchronize()
        else:
            # numpy copy: a torch op would drop and re-take the GIL around 33 KB
            h = host.numpy()
            np.copyto(h, self._gathered[slot].numpy())
            return h
        return host.numpy()


def pack_into(send: torch.Tensor, cls, prob) -> None:
    """Write host (cls int32 [n], prob fp32 [n]) into a send buffer slot."""
    c = np.ascontiguousarray(cls, np.int32)
    p = np.ascontiguousarray(prob, np.float32).view(np.int32)
    n = c.size
    if send.device.type == "cpu":
        s = send.numpy()                     # in place, without a GIL round-trip per torch op
        s[:n, 0] = c
        s[:n, 1] = p
        return
    send[:n, 0].copy_(torch.as_tensor(c).to(send.device))
    send[:n, 1].copy_(torch.as_tensor(p).to(send.device))
