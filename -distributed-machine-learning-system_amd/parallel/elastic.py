"""Epoch-versioned collective group for the fault-tolerant node runtime
(SURVEY.md §5.8 "RCCL fault tolerance", §7.3 hard part 2).

The steady-state query path of a healthy cluster runs in *rounds* on a
torch.distributed group ("nccl" == RCCL over xGMI on MI355X, "gloo" on CPU):
the coordinator (rank 0) broadcasts one descriptor row per member and gathers
the packed top-1 results — the same ``QueryPlane`` bench.py uses.  Membership
changes are handled by re-forming the group under a new *epoch*:

  * the coordinator announces GROUP_FORM {epoch, members, port} over the TCP
    control plane; every member tears down its previous process group
    (destroying it aborts RCCL communicators, so a collective blocked on a dead
    peer returns) and rendezvous on a fresh TCPStore hosted by the coordinator
    under the prefix ``epoch<N>``;
  * a round whose collectives fail (peer died mid-round) is abandoned; its
    chunks fall back to the TCP JOB path (idempotent results), and the
    coordinator re-forms the group over the survivors once the failure
    detector has removed the dead node.

Liveness is bounded by the failure detector, not by a collective timeout:
every collective is issued with ``async_op=True`` and polled in short slices
against a caller check (membership of the round's ranks, a newer epoch, node
shutdown).  A round whose check fails raises ``RoundAbandoned`` at once and
the communicator is aborted in the background (``_abort_process_group``:
ncclCommAbort on RCCL), so a dead rank costs ``failure_timeout_s`` plus the
re-form, never the process-group timeout -- which is therefore set long
(idle members may wait for the next round indefinitely).

Only one process group exists per process at a time (torch's default group);
a new epoch waits for the previous epoch's abort to finish.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from datetime import timedelta

import torch
import torch.distributed as dist

from .dataplane import NO_WORK, Env, QueryPlane

log = logging.getLogger("idunno.elastic")

MODEL_IDS = {"alexnet": 0, "resnet18": 1, "resnet50": 2, "resnet34": 3}
MODEL_NAMES = {v: k for k, v in MODEL_IDS.items()}
STOP = -2          # descriptor start value telling members to leave the round loop
IDLE_TIMEOUT = timedelta(hours=24)   # process-group timeout: liveness comes from the caller's check


class RoundAbandoned(RuntimeError):
    """A round's liveness check failed (dead rank, newer epoch, shutdown)."""


class ElasticGroup:
    def __init__(self, device: torch.device, backend: str | None = None, timeout_s: float = 30.0,
                 max_chunk: int = 1024):
        self.device = torch.device(device)
        self.backend = backend or ("nccl" if self.device.type == "cuda" else "gloo")
        self.timeout_s = timeout_s
        self.max_chunk = max_chunk
        self.epoch = -1
        self.members: list[str] = []
        self.rank = -1
        self.plane: QueryPlane | None = None
        self.lock = threading.RLock()
        self._store = None
        self._aborter: threading.Thread | None = None
        self.poll_s = 0.0005

    @property
    def formed(self) -> bool:
        return self.plane is not None

    def teardown(self) -> None:
        """Clean teardown of a healthy group (no collective in flight)."""
        with self.lock:
            self._join_aborter()
            self.plane = None
            if dist.is_initialized():
                try:
                    dist.destroy_process_group()
                except Exception:  # noqa: BLE001  (a broken group can fail to clean up)
                    log.exception("destroy_process_group failed")
            self._store = None

    def abort_async(self) -> None:
        """Abandon the current epoch with collectives possibly still pending:
        abort the communicator on a background thread (RCCL: ncclCommAbort
        returns at once; gloo returns once the peers' sockets close) so the
        caller never blocks on a dead peer."""
        with self.lock:
            if self.plane is None and not dist.is_initialized():
                return
            self.plane = None
            self._store = None

            def run():
                try:
                    if dist.is_initialized():
                        dist.distributed_c10d._abort_process_group()
                except Exception:  # noqa: BLE001
                    log.exception("abort of the old epoch failed")
                try:
                    if dist.is_initialized():
                        dist.destroy_process_group()
                except Exception:  # noqa: BLE001
                    pass

            self._join_aborter()
            self._aborter = threading.Thread(target=run, name="epoch-abort", daemon=True)
            self._aborter.start()

    def _join_aborter(self, timeout: float | None = None) -> bool:
        th = self._aborter
        if th is None:
            return True
        th.join(self.timeout_s if timeout is None else timeout)
        if th.is_alive():
            return False
        self._aborter = None
        return True

    def _wait(self, work, check) -> None:
        """Poll ``work`` until it completes; ``check()`` raises RoundAbandoned
        (liveness) between polls.  Spins ~1 ms, then sleeps ``poll_s``, backing
        off to 4x after 10 ms and 20x after 1 s of waiting (a member idling
        between queries wakes 100 times a second, not 2000; a round that
        follows a long idle gap pays at most ~10 ms more latency)."""
        if work is None:
            return
        t0 = time.perf_counter()
        while not work.is_completed():
            if check is not None:
                check()
            waited = time.perf_counter() - t0
            if waited > 0.001:
                time.sleep(self.poll_s * (1 if waited < 0.01 else 4 if waited < 1.0 else 20))
        work.wait()

    def form(self, me: str, members: list[str], epoch: int, host: str, port: int) -> bool:
        """Join epoch ``epoch`` of the group (blocking rendezvous).  Rank 0 is
        members[0], which hosts the TCPStore.  Returns False on failure."""
        with self.lock:
            if not self._join_aborter():
                log.warning("%s: previous epoch still aborting; cannot form epoch %d", me, epoch)
                return False
            self.teardown()
            if me not in members:
                return False
            rank = members.index(me)
            world = len(members)
            try:
                store = dist.TCPStore(host, port, world_size=world, is_master=(rank == 0),
                                      timeout=timedelta(seconds=self.timeout_s), wait_for_workers=False,
                                      use_libuv=False)
                pstore = dist.PrefixStore(f"epoch{epoch}", store)
                kw = {}
                if self.backend == "nccl":
                    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
                    kw["device_id"] = self.device
                # rendezvous / connection setup bounded by timeout_s; afterwards the
                # group's collectives may stay pending for an idle gap of any length
                dist.init_process_group(self.backend, store=pstore, rank=rank, world_size=world,
                                        timeout=timedelta(seconds=self.timeout_s), **kw)
                dist.distributed_c10d._set_pg_timeout(IDLE_TIMEOUT, None)
            except Exception:  # noqa: BLE001
                log.exception("%s: forming epoch %d failed", me, epoch)
                self._store = None
                return False
            self._store = store
            self.epoch, self.members, self.rank = epoch, list(members), rank
            env = Env(rank, world, self.device.index or 0, self.device, self.backend)
            self.plane = QueryPlane(env, coordinator=0, max_chunk=self.max_chunk)
            return True

    # -- one round ------------------------------------------------------------------
    def round(self, table: list[tuple[int, int, int, int]] | None, run_chunk, check=None):
        """Run one collective round.

        Rank 0 passes ``table`` (one (model_id, qnum, start, end) row per member,
        end = NO_WORK for idle members, start = STOP to end the round loop).
        Every member runs ``run_chunk(model, start, end, packed)`` on its row:
        it either writes (class, prob bits) pairs into the device send buffer
        ``packed`` itself and returns None (device-resident results), or returns
        (cls, prob) host arrays that are packed here.  The results are gathered
        to rank 0, which gets back ``[(row, cls np, prob np), ...]`` from ONE
        device->host copy; other ranks get None.  ``check()`` is polled while a
        collective is pending and raises RoundAbandoned to give up (the caller
        then calls ``abort_async``); any collective error also raises."""
        from .dataplane import unpack

        plane = self.plane
        if plane is None:
            raise RuntimeError("group not formed")
        self._wait(plane.dispatch_async(table), check)
        mid, qnum, s, e = plane.my_row()
        if s == STOP:
            return "stop"
        if e != NO_WORK:
            r = run_chunk(MODEL_NAMES[mid], s, e, plane.send_buffer)
            if r is not None:
                cls, prob = r
                plane.pack(torch.as_tensor(cls).to(self.device), torch.as_tensor(prob).to(self.device))
        self._wait(plane.gather_async(), check)
        if plane.env.rank != 0:
            return None
        allres = plane.gathered_all.cpu()
        out = []
        for r, row in enumerate(table):
            if row[3] == NO_WORK or row[2] == STOP:
                continue
            c, p = unpack(allres[r], row[3] - row[2] + 1)
            out.append((row, c.numpy(), p.numpy()))
        return out
