"""Opt-in race detector for the control-plane runtime.

The reference declares locks it never takes (``sdfs_lock``, ``jobs_lock``,
``mp4_machinelearning.py:122-124``), mutates its job-state tables from several
threads without any lock (``:529-533, 638-644, 714-754``) and acquires locks by
hand, so an exception between acquire and release leaves ``ml_lock`` held forever
(``:204-218``).  This module is the tool that keeps those bug classes out of this
runtime; it is off unless ``IDUNNO_RACECHECK`` is set, and then costs a dict
lookup per table access.

Two detectors:

* **Lockset (Eraser).**  ``instrument(obj, attrs)`` swaps the named container
  attributes for watched copies.  Each container starts *exclusive* to the first
  thread that touches it; once a second thread touches it, its candidate lockset
  is refined to the intersection of the tracked locks held at every access.  An
  empty lockset means two threads reached the table with no common lock: a data
  race, reported with both thread names and the offending call site.
* **Lock order.**  Every ``make_lock`` lock, when tracked, records an edge
  ``held -> acquired`` per acquisition; an acquisition that closes a cycle in that
  graph is a potential deadlock (the pair was taken in both orders), reported
  the first time it happens.

Reports accumulate in ``reports()``; ``IDUNNO_RACECHECK=raise`` turns the first one
into a ``RaceError`` at the access, and a non-empty list is printed at exit.
"""
from __future__ import annotations

import atexit
import itertools
import os
import sys
import threading
import traceback
from collections import defaultdict, deque

_MODE = os.environ.get("IDUNNO_RACECHECK", "").strip().lower()
_ENABLED = _MODE not in ("", "0", "off", "false")

_tls = threading.local()
_glock = threading.Lock()         # guards the detector's own state
_reports: list[str] = []
_edges: dict[int, set[int]] = defaultdict(set)
_names: dict[int, str] = {}
_reported_pairs: set = set()


class RaceError(RuntimeError):
    pass


def enabled() -> bool:
    return _ENABLED


def enable(on: bool = True, mode: str = "report") -> None:
    """Switch the detector at run time (tests).  Only locks and containers
    created while it is on are tracked."""
    global _ENABLED, _MODE
    _ENABLED, _MODE = bool(on), (mode if on else "")


def reports() -> list[str]:
    with _glock:
        return list(_reports)


def clear() -> None:
    with _glock:
        _reports.clear()
        _edges.clear()
        _names.clear()
        _reported_pairs.clear()


def _report(msg: str) -> None:
    site = "".join(traceback.format_stack(limit=6)[:-2])
    with _glock:
        _reports.append(f"{msg}\n{site}")
    if _MODE == "raise":
        raise RaceError(msg)


_tids = itertools.count(1)


def _tid() -> int:
    """Per-thread id that is never reused (OS thread idents are, once a thread
    exits, which would make a later thread look like the exclusive owner)."""
    t = getattr(_tls, "tid", None)
    if t is None:
        t = _tls.tid = next(_tids)
    return t


def _held() -> list:
    h = getattr(_tls, "held", None)
    if h is None:
        h = _tls.held = []
    return h


# -- lock-order tracking ---------------------------------------------------------
def _path(src: int, dst: int) -> bool:
    """Is dst reachable from src in the order graph?  (caller holds _glock)"""
    seen, todo = {src}, deque([src])
    while todo:
        u = todo.popleft()
        if u == dst:
            return True
        for v in _edges.get(u, ()):
            if v not in seen:
                seen.add(v)
                todo.append(v)
    return False


class TrackedLock:
    """``threading.Lock`` / ``RLock`` stand-in that knows its owner and feeds the
    lock-order graph.  Same ``acquire`` / ``release`` / context-manager API."""

    def __init__(self, name: str, reentrant: bool = False):
        self._lk = threading.RLock() if reentrant else threading.Lock()
        self.name = name
        self.reentrant = reentrant
        self._owner: int | None = None
        self._depth = 0
        with _glock:
            _names[id(self)] = name

    def held_by_me(self) -> bool:
        return self._owner == _tid()

    def _note_order(self) -> None:
        me = id(self)
        inversion = None
        with _glock:
            for h in _held():
                hid = id(h)
                if hid == me or me in _edges[hid]:
                    continue
                if _path(me, hid) and (me, hid) not in _reported_pairs:
                    _reported_pairs.add((me, hid))
                    _reported_pairs.add((hid, me))
                    inversion = (h.name, self.name)
                _edges[hid].add(me)
        if inversion:
            _report(f"lock-order inversion: {inversion[1]!r} acquired while holding {inversion[0]!r}, "
                    f"but {inversion[1]!r} -> {inversion[0]!r} was seen before (potential deadlock) "
                    f"[thread {threading.current_thread().name}]")

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        if not (self.reentrant and self.held_by_me()):
            self._note_order()
        ok = self._lk.acquire(blocking, timeout)
        if ok:
            if self._depth == 0:
                self._owner = _tid()
                _held().append(self)
            self._depth += 1
        return ok

    def release(self) -> None:
        if not self.held_by_me():
            _report(f"lock {self.name!r} released by thread {threading.current_thread().name} "
                    f"that does not hold it")
        self._depth -= 1
        if self._depth == 0:
            self._owner = None
            h = _held()
            for i in range(len(h) - 1, -1, -1):
                if h[i] is self:
                    del h[i]
                    break
        self._lk.release()

    def locked(self) -> bool:
        return self._owner is not None

    __enter__ = acquire

    def __exit__(self, *exc) -> None:
        self.release()


def make_lock(name: str, reentrant: bool = False):
    """The runtime's lock factory: a plain ``threading`` lock normally, a
    ``TrackedLock`` when the detector is on."""
    if _ENABLED:
        return TrackedLock(name, reentrant)
    return threading.RLock() if reentrant else threading.Lock()


def assert_held(lock, what: str = "") -> None:
    """Check (when tracking) that the calling thread holds ``lock``; for helpers
    documented as 'caller holds the lock'."""
    if isinstance(lock, TrackedLock) and not lock.held_by_me():
        _report(f"{what or 'guarded section'} entered without holding {lock.name!r} "
                f"[thread {threading.current_thread().name}]")


# -- lockset (Eraser) tracking ---------------------------------------------------
class _Shadow:
    __slots__ = ("name", "owner", "owner_name", "lockset", "reported", "last")

    def __init__(self, name: str):
        self.name = name
        self.owner: int | None = None
        self.owner_name = ""
        self.lockset: set[int] | None = None   # None while exclusive
        self.reported = False
        self.last = ""

    def access(self) -> None:
        if self.reported:
            return
        me, cur = _tid(), threading.current_thread().name
        prev, self.last = self.last, cur
        if self.owner is None:
            self.owner, self.owner_name = me, cur
            return
        if self.lockset is None:
            if me == self.owner:
                return
            self.lockset = {id(h) for h in _held()}        # first shared access
            prev = self.owner_name
        else:
            self.lockset &= {id(h) for h in _held()}
        if not self.lockset:
            self.reported = True
            _report(f"data race on {self.name}: thread {cur} accessed it with no lock in common with "
                    f"earlier accesses (previous: thread {prev}, first owner: {self.owner_name})")


def _watched(base):
    class Watched(base):
        __slots__ = ("_rc",)
    for meth in ("__getitem__", "__setitem__", "__delitem__", "__contains__", "__iter__", "__len__",
                 "get", "setdefault", "pop", "popitem", "update", "clear", "items", "keys", "values",
                 "append", "extend", "remove", "insert", "add", "discard", "appendleft", "popleft",
                 "__missing__"):
        f = getattr(base, meth, None)
        if f is None:
            continue

        def wrap(f=f):
            def g(self, *a, **k):
                rc = getattr(self, "_rc", None)
                if rc is not None:
                    rc.access()
                return f(self, *a, **k)
            g.__name__ = f.__name__
            return g
        setattr(Watched, meth, wrap())
    Watched.__name__ = f"Watched{base.__name__}"
    return Watched


_WATCHED: dict = {}


def watch(container, name: str):
    """A watched copy of a dict / defaultdict / list / set / deque."""
    base = type(container)
    cls = _WATCHED.get(base)
    if cls is None:
        cls = _WATCHED[base] = _watched(base)
    if base.__name__ == "defaultdict":
        w = cls(container.default_factory, container)
    elif base is deque:
        w = cls(container, container.maxlen)
    else:
        w = cls(container)
    w._rc = _Shadow(name)
    return w


def instrument(obj, attrs, owner: str | None = None) -> None:
    """Replace ``obj.<attr>`` containers by watched copies (no-op when off).
    Call again after code that rebinds the attributes (e.g. a snapshot restore)."""
    if not _ENABLED:
        return
    tag = owner or type(obj).__name__
    for a in attrs:
        v = getattr(obj, a)
        if getattr(v, "_rc", None) is None:
            setattr(obj, a, watch(v, f"{tag}.{a}"))


@atexit.register
def _dump() -> None:
    if _ENABLED and _reports:
        sys.stderr.write(f"[racecheck] {len(_reports)} report(s):\n" + "\n".join(_reports) + "\n")
