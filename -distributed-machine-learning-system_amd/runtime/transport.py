"""Control-plane transports (SURVEY.md §2.5 M1-M13, §5.8 "control plane = host IPC").

Two interchangeable implementations of one small interface:

  * ``TcpTransport``     length-prefixed msgpack frames over persistent
                         localhost TCP connections (one listening port per
                         node); used by the multi-process node runtime.
  * ``InMemoryNetwork``  all nodes in one process, with injectable message
                         drop, delay, partitions and node crashes; used by the
                         fake multi-node tests (SURVEY.md §4 "fake transport").

Interface: ``start(handler)``, ``send(dst, msg) -> bool`` (False = peer
unreachable, the analogue of a refused connect), ``request(dst, msg,
timeout) -> reply`` (rid-matched REPLY frame), ``close()``.  Handlers run on a
small per-node thread pool so a long handler (an inference chunk, an SDFS
transfer) never blocks the receive path.
"""
from __future__ import annotations

import ctypes
import errno
import itertools
import logging
import random
import socket
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from concurrent.futures import TimeoutError as FuturesTimeout

from .messages import FrameReader, Type, encode

log = logging.getLogger("idunno.transport")


# Frames go out through libc ``send`` called via a PyDLL handle, i.e. WITHOUT
# releasing the GIL, and with MSG_DONTWAIT: a control frame to a localhost peer
# fits the socket buffer and is copied in a few microseconds.  ``socket.sendall``
# releases and re-acquires the GIL around every call, and on a busy host each
# re-acquire can queue behind the node's other threads (receivers, heartbeats,
# the round loop): a 7-peer multicast paid that convoy seven times.  A send
# that would block (full buffer) finishes through ``sendall`` as before.
try:
    _LIBC = ctypes.PyDLL(None, use_errno=True)
    _SEND = _LIBC.send
    _SEND.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    _SEND.restype = ctypes.c_ssize_t
except (OSError, AttributeError):          # pragma: no cover - non-glibc host
    _SEND = None
_MSG_DONTWAIT, _MSG_NOSIGNAL = 0x40, 0x4000


def _send_frame(sock: socket.socket, data: bytes) -> None:
    """``sock.sendall(data)``, holding the GIL for the common non-blocking case."""
    n = 0
    if _SEND is not None and type(data) is bytes:
        n = _SEND(sock.fileno(), data, len(data), _MSG_DONTWAIT | _MSG_NOSIGNAL)
        if n == len(data):
            return
        if n < 0:
            e = ctypes.get_errno()
            if e not in (errno.EAGAIN, errno.EWOULDBLOCK, errno.EINTR):
                raise OSError(e, "send failed")
            n = 0
    sock.sendall(memoryview(data)[n:])


class TransportError(RuntimeError):
    pass


class BaseTransport:
    def __init__(self, name: str, workers: int = 8):
        self.name = name
        self.handler = None
        self._pool = ThreadPoolExecutor(max_workers=workers, thread_name_prefix=f"{name}-h")
        self._rid = itertools.count(1)
        self._pending: dict[int, Future] = {}
        self._plock = threading.Lock()
        self.closed = False
        self.dead_check = None          # optional f(dst) -> True once the FD declares dst dead

    # subclasses implement _send_raw(dst, msg) -> bool
    def _send_raw(self, dst: str, msg: dict) -> bool:  # pragma: no cover
        raise NotImplementedError

    def start(self, handler) -> None:
        self.handler = handler

    def send(self, dst: str, msg: dict) -> bool:
        if self.closed:
            return False
        msg.setdefault("src", self.name)
        return self._send_raw(dst, msg)

    def multicast(self, dsts, msg: dict) -> list[str]:
        """Send one message to several peers; returns the peers it did not
        reach.  TCP encodes the frame once and writes the same bytes to every
        link (a round's descriptor table goes to all members this way)."""
        if self.closed:
            return list(dsts)
        msg.setdefault("src", self.name)
        return [d for d in dsts if not self._send_raw(d, msg)]

    def request(self, dst: str, msg: dict, timeout: float = 5.0) -> dict:
        rid = next(self._rid)
        fut: Future = Future()
        with self._plock:
            self._pending[rid] = fut
        msg = dict(msg, rid=rid, src=self.name)
        try:
            if not self._send_raw(dst, msg):
                raise TransportError(f"{dst} unreachable")
            # wait in slices so a peer the failure detector declares dead fails
            # the call at once instead of holding the caller for the full timeout
            end = time.monotonic() + timeout
            while True:
                left = end - time.monotonic()
                if left <= 0:
                    raise FuturesTimeout()
                try:
                    return fut.result(timeout=min(left, 0.05))
                except (TimeoutError, FuturesTimeout):
                    if self.dead_check is not None and self.dead_check(dst):
                        raise TransportError(f"{dst} declared dead while waiting for {msg.get('t')}")
        except (TimeoutError, FuturesTimeout) as e:
            raise TransportError(f"request {msg.get('t')} to {dst} timed out") from e
        finally:
            with self._plock:
                self._pending.pop(rid, None)

    def _deliver(self, msg: dict) -> None:
        """Called by the receive path for every decoded frame."""
        if msg.get("t") == Type.REPLY:
            with self._plock:
                fut = self._pending.get(msg.get("rid"))
            if fut is not None and not fut.done():
                fut.set_result(msg)
            return
        if self.closed or self.handler is None:
            return
        try:
            self._pool.submit(self._run_handler, msg)
        except RuntimeError:  # pool shut down
            pass

    def _run_handler(self, msg: dict) -> None:
        try:
            reply = self.handler(msg)
        except Exception as e:  # noqa: BLE001
            log.exception("%s: handler failed on %s", self.name, msg.get("t"))
            reply = {"ok": False, "error": f"{type(e).__name__}: {e}"}
        if "rid" in msg and msg.get("src"):
            if reply is None:
                reply = {"ok": True}
            reply = dict(reply, t=Type.REPLY, rid=msg["rid"], src=self.name)
            self._send_raw(msg["src"], reply)

    def close(self) -> None:
        self.closed = True
        self._pool.shutdown(wait=False, cancel_futures=True)
        with self._plock:
            for f in self._pending.values():
                if not f.done():
                    f.set_exception(TransportError("transport closed"))


# ---------------------------------------------------------------------------
# in-memory network with fault injection
# ---------------------------------------------------------------------------

class InMemoryNetwork:
    """A fake network for N nodes in one process.

    Fault knobs: ``drop_rate`` (random loss), ``delay_s`` (fixed latency),
    ``partition(a, b)`` (bidirectional cut), ``crash(node)`` (node stops
    sending and receiving; sends to it fail like a refused connect).
    """

    def __init__(self, drop_rate: float = 0.0, delay_s: float = 0.0, seed: int = 0):
        self.nodes: dict[str, InMemoryTransport] = {}
        self.drop_rate = drop_rate
        self.delay_s = delay_s
        self.cut: set = set()
        self.crashed: set = set()
        self.rng = random.Random(seed)
        self.lock = threading.Lock()
        self.sent = 0

    def transport(self, name: str) -> "InMemoryTransport":
        t = InMemoryTransport(name, self)
        self.nodes[name] = t
        self.crashed.discard(name)
        return t

    def partition(self, a: str, b: str) -> None:
        self.cut |= {(a, b), (b, a)}

    def heal(self) -> None:
        self.cut.clear()

    def crash(self, name: str) -> None:
        self.crashed.add(name)

    def route(self, src: str, dst: str, msg: dict) -> bool:
        with self.lock:
            self.sent += 1
            if src in self.crashed:
                return False
            t = self.nodes.get(dst)
            if t is None or dst in self.crashed or t.closed:
                return False
            if (src, dst) in self.cut:
                return True  # silently lost, like a partition
            if self.drop_rate and self.rng.random() < self.drop_rate:
                return True
        # deep-ish copy semantics: the receiver must not alias sender state
        import msgpack

        m = msgpack.unpackb(msgpack.packb(msg, use_bin_type=True), raw=False, strict_map_key=False)
        if self.delay_s:
            threading.Timer(self.delay_s, t._deliver, args=(m,)).start()
        else:
            t._deliver(m)
        return True


class InMemoryTransport(BaseTransport):
    def __init__(self, name: str, net: InMemoryNetwork):
        super().__init__(name)
        self.net = net

    def _send_raw(self, dst: str, msg: dict) -> bool:
        return self.net.route(self.name, dst, msg)


# ---------------------------------------------------------------------------
# TCP
# ---------------------------------------------------------------------------

class TcpTransport(BaseTransport):
    """Persistent localhost TCP links, one listener per node."""

    def __init__(self, name: str, addr_of, bind: tuple[str, int], connect_timeout: float = 1.0):
        super().__init__(name)
        self.addr_of = addr_of                 # callable: node name -> (host, port)
        self.bind = bind
        self.connect_timeout = connect_timeout
        self._out: dict[str, socket.socket] = {}
        self._out_locks: dict[str, threading.Lock] = {}
        self._in: set = set()
        self._olock = threading.Lock()
        self._srv: socket.socket | None = None
        self._threads: list[threading.Thread] = []

    def start(self, handler) -> None:
        super().start(handler)
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind(self.bind)
        srv.listen(64)
        self._srv = srv
        th = threading.Thread(target=self._accept_loop, name=f"{self.name}-accept", daemon=True)
        th.start()
        self._threads.append(th)

    def _accept_loop(self) -> None:
        while not self.closed:
            try:
                conn, _ = self._srv.accept()
            except OSError:
                return
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            with self._olock:
                self._in.add(conn)
            threading.Thread(target=self._read_loop, args=(conn,), daemon=True,
                             name=f"{self.name}-rx").start()

    def _read_loop(self, conn: socket.socket) -> None:
        rd = FrameReader()
        try:
            while not self.closed:
                data = conn.recv(1 << 20)
                if not data:
                    break
                for m in rd.feed(data):
                    self._deliver(m)
        except OSError:
            pass
        finally:
            with self._olock:
                self._in.discard(conn)
            conn.close()

    def _conn(self, dst: str) -> socket.socket:
        with self._olock:
            s = self._out.get(dst)
            if s is not None:
                return s
        s = socket.create_connection(self.addr_of(dst), timeout=self.connect_timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.settimeout(None)
        with self._olock:
            old = self._out.get(dst)
            if old is not None:
                s.close()
                return old
            self._out[dst] = s
            return s

    def _drop(self, dst: str) -> None:
        with self._olock:
            s = self._out.pop(dst, None)
        if s is not None:
            try:
                s.close()
            except OSError:
                pass

    def multicast(self, dsts, msg: dict) -> list[str]:
        if self.closed:
            return list(dsts)
        msg.setdefault("src", self.name)
        data = encode(msg)
        return [d for d in dsts if not self._send_bytes(d, data)]

    def _send_raw(self, dst: str, msg: dict) -> bool:
        return self._send_bytes(dst, encode(msg))

    def _send_bytes(self, dst: str, data: bytes) -> bool:
        with self._olock:
            lk = self._out_locks.setdefault(dst, threading.Lock())
        with lk:
            for attempt in (0, 1):
                try:
                    _send_frame(self._conn(dst), data)
                    return True
                except OSError:
                    self._drop(dst)
                    if attempt:
                        return False
        return False

    def close(self) -> None:
        super().close()
        if self._srv is not None:
            try:
                self._srv.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            self._srv.close()
        with self._olock:
            for s in list(self._out.values()) + list(self._in):
                try:
                    s.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                try:
                    s.close()
                except OSError:
                    pass
            self._out.clear()
            self._in.clear()


def wait_for(pred, timeout: float, interval: float = 0.01) -> bool:
    """Poll ``pred`` until it is true or ``timeout`` elapses."""
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(interval)
    return bool(pred())
