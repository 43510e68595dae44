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

Only one process group exists per process at a time (torch's default group).
"""
from __future__ import annotations

import logging
import os
import threading
from datetime import timedelta

import torch
import torch.distributed as dist

from .dataplane import NO_WORK, Env, QueryPlane

log = logging.getLogger("idunno.elastic")

MODEL_IDS = {"alexnet": 0, "resnet18": 1, "resnet50": 2, "resnet34": 3}
MODEL_NAMES = {v: k for k, v in MODEL_IDS.items()}
STOP = -2          # descriptor start value telling members to leave the round loop


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

    @property
    def formed(self) -> bool:
        return self.plane is not None

    def teardown(self) -> None:
        with self.lock:
            self.plane = None
            if dist.is_initialized():
                try:
                    dist.destroy_process_group()
                except Exception:  # noqa: BLE001  (a broken group can fail to clean up)
                    log.exception("destroy_process_group failed")
            self._store = None

    def form(self, me: str, members: list[str], epoch: int, host: str, port: int) -> bool:
        """Join epoch ``epoch`` of the group (blocking rendezvous).  Rank 0 is
        members[0], which hosts the TCPStore.  Returns False on failure."""
        with self.lock:
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
                dist.init_process_group(self.backend, store=pstore, rank=rank, world_size=world,
                                        timeout=timedelta(seconds=self.timeout_s), **kw)
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
    def round(self, table: list[tuple[int, int, int, int]] | None, run_chunk):
        """Run one collective round.

        Rank 0 passes ``table`` (one (model_id, qnum, start, end) row per member,
        end = NO_WORK for idle members, start = STOP to end the round loop).
        Every member runs ``run_chunk(model, start, end) -> (cls, prob)`` on its
        row and the packed results are gathered to rank 0, which gets back
        ``[(row, cls np, prob np), ...]``; other ranks get None.  Raises on any
        collective failure (the caller abandons the round and re-forms)."""
        from .dataplane import unpack

        plane = self.plane
        if plane is None:
            raise RuntimeError("group not formed")
        mid, qnum, s, e = plane.dispatch(table)
        if s == STOP:
            return "stop"
        if e != NO_WORK:
            cls, prob = run_chunk(MODEL_NAMES[mid], s, e)
            cls_t = torch.as_tensor(cls).to(self.device)
            prob_t = torch.as_tensor(prob).to(self.device)
        else:
            cls_t = torch.zeros(0, dtype=torch.int32, device=self.device)
            prob_t = torch.zeros(0, dtype=torch.float32, device=self.device)
        got = plane.gather(cls_t, prob_t)
        if plane.env.rank != 0:
            return None
        out = []
        for r, row in enumerate(table):
            if row[3] == NO_WORK or row[2] == STOP:
                continue
            c, p = unpack(got[r].cpu(), row[3] - row[2] + 1)
            out.append((row, c.numpy(), p.numpy()))
        return out
