"""Membership list + heartbeat failure detector.

Reference behaviour kept:
  * the acting master (the coordinator) PINGs every member every
    ``heartbeat_period_s`` (0.3 s) with its full membership list; members
    merge it (LEAVE overrides, otherwise the newer timestamp wins,
    mp4_machinelearning.py:272-282) and answer PONG with their own entry;
  * a member with no PONG for ``failure_timeout_s`` (2 s) is marked LEAVE
    and the failure callbacks run (SDFS re-replication, chunk re-dispatch);
  * JOIN goes to the introducer (the master), which adds the joiner and
    forwards the JOIN to everyone else; ``leave`` stops answering.

Added (the reference has no coordinator failure detection, C9 stub):
  * every member records the last PING from the master; the hot standby
    treats ``failure_timeout_s`` without one as a master failure and promotes
    itself (``on_master_failure``), announcing a higher ``epoch``;
  * members follow the master with the highest epoch they have seen, so a
    stale master that comes back is ignored;
  * ``leave`` also sends an explicit LEAVE so voluntary departures are seen
    at once (and rejoin works with a fresh timestamp).
Single lock, exception-safe (fix A13); one ping thread instead of nine.
"""
from __future__ import annotations

import logging
import threading
import time

from ..utils import racecheck
from .messages import Status_LEAVE, Status_RUNNING, Type

log = logging.getLogger("idunno.membership")


class Membership:
    def __init__(self, name: str, cfg, transport, master: str, clock=time.monotonic,
                 wall=time.time):
        self.name = name
        self.cfg = cfg
        self.t = transport
        self.clock = clock
        self.wall = wall
        self.lock = racecheck.make_lock("membership", reentrant=True)
        self.members: dict[str, list] = {}
        self.master = master
        self.epoch = 0
        self.joined = False
        self.left = False
        self.last_ack: dict[str, float] = {}
        self.last_master_ping = clock()
        self.on_failure: list = []          # f(node)
        self.on_join: list = []             # f(node)
        self.on_master_failure: list = []   # f(old_master)
        self.on_master_change: list = []    # f(new_master, epoch)
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self.master_suspected = False
        racecheck.instrument(self, ("members", "last_ack"), f"Membership[{name}]")

    # -- views ----------------------------------------------------------------
    def is_master(self) -> bool:
        return self.master == self.name

    def alive(self) -> list[str]:
        with self.lock:
            return sorted(n for n, (_, st) in self.members.items() if st == Status_RUNNING)

    def is_alive(self, node: str) -> bool:
        with self.lock:
            e = self.members.get(node)
            return e is not None and e[1] == Status_RUNNING

    def self_id(self) -> str:
        """Reference list_self: ``IP#timestamp`` (:1062-1068)."""
        with self.lock:
            e = self.members.get(self.name)
        ts = e[0] if e else 0.0
        host, port = self.cfg.address(self.name)
        return f"{host}:{port}#{ts}"

    def table(self) -> dict:
        with self.lock:
            return {k: list(v) for k, v in self.members.items()}

    # -- lifecycle ------------------------------------------------------------
    def start(self) -> None:
        for fn, nm in ((self._ping_loop, "ping"), (self._monitor_loop, "monitor")):
            th = threading.Thread(target=fn, name=f"{self.name}-{nm}", daemon=True)
            th.start()
            self._threads.append(th)

    def stop(self) -> None:
        self._stop.set()

    def join(self, timeout: float = 3.0) -> bool:
        """Join through the introducer (the current master)."""
        now = self.wall()
        with self.lock:
            self.left = False
            self.members[self.name] = [now, Status_RUNNING]
        self.last_master_ping = self.clock()
        if self.is_master():
            self.joined = True
            return True
        try:
            rep = self.t.request(self.master, {"t": Type.JOIN, "entry": [now, Status_RUNNING]}, timeout)
        except Exception as e:  # noqa: BLE001
            log.warning("%s: join via %s failed: %s", self.name, self.master, e)
            return False
        self.last_master_ping = self.clock()
        self.joined = True
        self._merge(rep.get("members", {}))
        with self.lock:
            if rep.get("epoch", 0) >= self.epoch:
                self.epoch = rep.get("epoch", 0)
        return True

    def leave(self) -> None:
        with self.lock:
            e = self.members.get(self.name, [self.wall(), Status_RUNNING])
            self.members[self.name] = [e[0], Status_LEAVE]
            self.left = True
            self.joined = False
        if not self.is_master():
            self.t.send(self.master, {"t": Type.LEAVE})

    # -- master side ------------------------------------------------------------
    def add_member(self, node: str, entry) -> None:
        fresh = False
        with self.lock:
            cur = self.members.get(node)
            if cur is None or cur[1] != Status_RUNNING or entry[0] > cur[0]:
                fresh = cur is None or cur[1] != Status_RUNNING
                self.members[node] = [entry[0], Status_RUNNING]
            self.last_ack[node] = self.clock()
        if fresh:
            for cb in self.on_join:
                cb(node)

    def mark_failed(self, node: str) -> None:
        with self.lock:
            e = self.members.get(node)
            if e is None or e[1] == Status_LEAVE:
                return
            self.members[node] = [e[0], Status_LEAVE]
            self.last_ack.pop(node, None)
        log.warning("%s: %s marked LEAVE (failure detected)", self.name, node)
        for cb in self.on_failure:
            try:
                cb(node)
            except Exception:  # noqa: BLE001
                log.exception("failure callback")

    def become_master(self, epoch: int) -> None:
        with self.lock:
            self.master = self.name
            self.epoch = epoch
            now = self.clock()
            for n in self.members:
                self.last_ack[n] = now
        for cb in self.on_master_change:
            cb(self.name, epoch)

    def _ping_loop(self) -> None:
        while not self._stop.wait(self.cfg.heartbeat_period_s):
            if not self.is_master() or self.left:
                continue
            with self.lock:
                targets = [n for n, (_, st) in self.members.items() if st == Status_RUNNING and n != self.name]
                payload = {"t": Type.PING, "members": self.table(), "epoch": self.epoch}
            for n in targets:
                self.t.send(n, dict(payload))

    def _monitor_loop(self) -> None:
        period = min(self.cfg.heartbeat_period_s, 0.1)
        while not self._stop.wait(period):
            now = self.clock()
            if self.is_master() and not self.left:
                with self.lock:
                    dead = [n for n, (_, st) in self.members.items()
                            if st == Status_RUNNING and n != self.name
                            and now - self.last_ack.setdefault(n, now) > self.cfg.failure_timeout_s]
                for n in dead:
                    self.mark_failed(n)
            elif self.joined and not self.left:
                if now - self.last_master_ping > self.cfg.failure_timeout_s and not self.master_suspected:
                    self.master_suspected = True
                    old = self.master
                    log.warning("%s: no PING from master %s for %.1fs", self.name, old,
                                now - self.last_master_ping)
                    for cb in self.on_master_failure:
                        try:
                            cb(old)
                        except Exception:  # noqa: BLE001
                            log.exception("master-failure callback")

    # -- message handling ---------------------------------------------------------
    def _merge(self, members: dict) -> None:
        with self.lock:
            for n, (ts, st) in members.items():
                if n == self.name:
                    continue
                cur = self.members.get(n)
                if cur is None:
                    self.members[n] = [ts, st]
                elif st == Status_LEAVE and ts >= cur[0]:
                    self.members[n] = [ts, st]
                elif ts > cur[0]:
                    self.members[n] = [ts, st]

    def handle(self, msg: dict):
        t = msg["t"]
        src = msg.get("src")
        if t == Type.PING:
            if self.left:
                return None                            # a left node stays silent
            with self.lock:
                ep = msg.get("epoch", 0)
                if ep < self.epoch:
                    return None                        # stale master
                if src != self.master or ep > self.epoch:
                    self.master, self.epoch = src, ep
                    changed = True
                else:
                    changed = False
                self.last_master_ping = self.clock()
                self.master_suspected = False
            if changed:
                for cb in self.on_master_change:
                    cb(src, ep)
            self._merge(msg.get("members", {}))
            with self.lock:
                mine = self.members.get(self.name, [self.wall(), Status_RUNNING])
            self.t.send(src, {"t": Type.PONG, "entry": mine, "epoch": self.epoch})
            return None
        if t == Type.PONG:
            if self.is_master():
                with self.lock:
                    self.last_ack[src] = self.clock()
                    cur = self.members.get(src)
                    ent = msg.get("entry")
                    if cur is not None and ent and ent[1] == Status_RUNNING and cur[1] == Status_RUNNING:
                        cur[0] = max(cur[0], ent[0])
            return None
        if t == Type.JOIN:
            entry = msg.get("entry", [self.wall(), Status_RUNNING])
            if self.is_master():
                self.add_member(src, entry)
                with self.lock:
                    others = [n for n, (_, st) in self.members.items()
                              if st == Status_RUNNING and n not in (self.name, src)]
                for n in others:                       # forward the JOIN (reference :262-267)
                    self.t.send(n, {"t": Type.JOIN, "who": src, "entry": entry, "fwd": True})
                return {"ok": True, "members": self.table(), "epoch": self.epoch}
            who = msg.get("who", src)
            self._merge({who: entry})
            return {"ok": True}
        if t == Type.LEAVE:
            if self.is_master():
                self.mark_failed(src)
            return None
        if t == Type.PROMOTE:
            with self.lock:
                ep = msg.get("epoch", 0)
                if ep <= self.epoch and src == self.master:
                    return None
                if ep < self.epoch:
                    return None
                self.master, self.epoch = src, ep
                self.last_master_ping = self.clock()
                self.master_suspected = False
            for cb in self.on_master_change:
                cb(src, ep)
            return {"ok": True}
        return None
