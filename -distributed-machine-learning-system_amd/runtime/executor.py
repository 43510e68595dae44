"""Inference executors (layer L4; reference ``alexnet_resnet.deeplearning``,
alexnet_resnet.py:12-92).

The reference reloads the model from torch.hub on every chunk and runs batch-1
forwards (A6).  An executor here holds each model resident (weights built
once, BN-folded, in HBM) and runs the whole chunk as one batch:

  * ``HipExecutor``   the MI355X path: HIP kernels, one hipGraph per
                      (model, batch) replayed for every chunk;
  * ``TorchExecutor`` fp32 PyTorch reference modules (CPU hosts, tests);
  * ``FakeExecutor``  deterministic answers from the image index, no compute
                      (control-plane tests).
All return ``(cls int32 [n], prob float32 [n])`` numpy arrays.
"""
from __future__ import annotations

import logging
import threading
import time

import numpy as np
import torch

from ..models import reference as ref
from .data import is_resident

log = logging.getLogger("idunno.executor")


class Done:
    """An already finished ``Executor.submit`` (synchronous executors)."""

    synchronous = True           # the chunk ran inside submit() (the node times that call)

    def __init__(self, res):
        self._res = res

    def result(self):
        return self._res


class Executor:
    device = torch.device("cpu")

    def run(self, model: str, images: torch.Tensor | None, start: int, end: int):
        raise NotImplementedError

    def submit(self, model: str, images: torch.Tensor | None, start: int, end: int):
        """Start a chunk; ``.result()`` of the returned handle gives what
        ``run`` returns.  Asynchronous executors let the node's worker launch
        chunk k+1 before it post-processes chunk k."""
        return Done(self.run(model, images, start, end))

    def warmup(self, model: str, batch: int) -> None:
        pass


class FakeExecutor(Executor):
    def __init__(self, delay_per_image_s: float = 0.0):
        self.delay = delay_per_image_s
        self.calls = 0

    def run(self, model, images, start, end):
        self.calls += 1
        n = end - start + 1
        if self.delay:
            time.sleep(self.delay * n)
        idx = np.arange(start, end + 1, dtype=np.int64)
        salt = 7 if ref.canonical(model) == "alexnet" else 13
        return ((idx * 7919 + salt) % 1000).astype(np.int32), np.full(n, 0.5, dtype=np.float32)


class TorchExecutor(Executor):
    def __init__(self, device="cpu", seed: int = 0):
        self.device = torch.device(device)
        self.seed = seed
        self.models: dict[str, torch.nn.Module] = {}
        self.lock = threading.Lock()

    def _model(self, name):
        name = ref.canonical(name)
        with self.lock:
            m = self.models.get(name)
            if m is None:
                m = ref.build(name, seed=self.seed).to(self.device)
                self.models[name] = m
        return m

    @torch.no_grad()
    def run(self, model, images, start, end):
        m = self._model(model)
        x = ref.preprocess_u8(images.to(self.device))
        p = torch.softmax(m(x), dim=1)
        prob, cls = p.max(dim=1)
        return cls.to(torch.int32).cpu().numpy(), prob.float().cpu().numpy()


class _HipPending:
    def __init__(self, ex, slot, ev, out, model=None, images=None):
        self.ex, self.slot, self.ev, self.out = ex, slot, ev, out
        self.model, self.images = model, images
        self._res = None

    def result(self):
        if self._res is None:
            try:
                self.ev.synchronize()
                out = self.out
                self._res = (out[:, 0].numpy().copy(), out[:, 1].contiguous().view(torch.float32).numpy().copy())
            finally:
                self.ex._release(self.slot)
            if self.images is not None and (self._res[0] < 0).any():
                # the split range guard tripped (class -2): this chunk again on the
                # all-f32 kernels, which have fp32's range
                self._res = self.ex.rerun_exact(self.model, self.images)
            self.images = None
        return self._res


class HipExecutor(Executor):
    """gfx950 kernels; per-(model, batch) hipGraphs, weights resident in HBM.

    ``dtype`` "fp32" runs the reference-precision path (f32-input MFMA), "fp16"
    the f16-MFMA path.  Thread-safe: the TCP worker loop and the collective
    round driver of a node may call ``run`` / ``run_packed`` at the same time
    (a TCP re-dispatch next to a round chunk of the same model and size); the
    static graph input, the replay and the result read-back of one call are
    one critical section (results of two chunks must never mix)."""

    def __init__(self, device="cuda", seed: int = 0, use_graphs: bool = True, max_graphs: int = 16,
                 dtype: str = "fp32", fp32_impl: str = "split"):
        from .. import ops
        from ..models import HipRunner, build_program

        ops.load()  # loud failure if the extension is missing on a GPU host
        self.device = torch.device(device)
        self.seed = seed
        self.dtype = dtype
        self.asynchronous = True        # run_packed returns before the GPU finishes
        if fp32_impl not in ("split", "f32mfma"):
            raise ValueError(f"fp32_impl must be 'split' or 'f32mfma', got {fp32_impl!r}")
        self.fp32_impl = fp32_impl      # fp32 programs: split-fp16 kernels or the all-f32-MFMA kernels
        self.use_graphs = use_graphs
        self.max_graphs = max_graphs
        self._HipRunner, self._build = HipRunner, build_program
        self.runners: dict[str, object] = {}
        self._pool = None
        self.graphs_broken = False      # a capture failed: eager forwards only (see _capture)
        self.trim_ok = None             # callable(need) -> bool: may empty_cache run now (see _capture)
        self._trim_wanted = False       # a new capture's trim is still owed (maybe_trim)
        self.trim_slack_bytes = 16 << 30      # reserved-but-unused cache that counts as a need to trim
        self.lock = threading.Lock()
        self.run_lock = threading.Lock()      # one forward (copy-in, replay, read-back) at a time
        self.stream = None      # private HIP stream: nodes sharing a GPU overlap
        # two launch slots (graph set + pinned result buffer each): a chunk can
        # run while the previous one's results are read back and ingested
        self._slots = [None, None]                      # pinned [>= n, 2] int32 per slot
        self._slot_busy = [False, False]
        self._slot_cv = threading.Condition()
        self._next_slot = 0
        self.closed = False

    def runner(self, name):
        name = ref.canonical(name)
        with self.lock:
            r = self.runners.get(name)
            if r is None:
                with torch.cuda.device(self.device):
                    r = self._HipRunner(self._build(name, seed=self.seed, dtype=self.dtype), self.device)
                    r.split = self.fp32_impl == "split"
                    # every graph of this executor replays on its one private stream and
                    # its outputs are read (D2H / the caller's packed buffer) before the
                    # next replay: one memory pool for all of them, so graph memory is
                    # the largest graph's, not the sum over chunk sizes (8 node
                    # processes sharing one GPU ran out of its 288 GB with a pool per
                    # graph once the fair-time split re-planned chunk sizes, round 6)
                    if self._pool is None:
                        self._pool = torch.cuda.graph_pool_handle()
                    r.graph_pool = self._pool
                self.runners[name] = r
        return r

    def warmup(self, model, batch):
        if self.use_graphs:
            with torch.cuda.device(self.device), self.run_lock:
                self.runner(model).capture(batch)

    def _can_capture(self, r) -> bool:
        return not self.closed and self.use_graphs and not self.graphs_broken and len(r._graphs) < self.max_graphs

    def _capture(self, r, fn):
        """Run a graph lookup / capture ``fn``.  A NEW capture is followed by
        ``empty_cache``: its eager warm-up forwards left activation blocks of
        that chunk size cached outside the graph pool, and with chunk sizes that
        move with the fair-time split those blocks pile up (8 node processes on
        one GPU: 20 GB reserved-but-unused each).  A capture that fails (e.g.
        out of memory) leaves the pool it recorded into unusable: the runners
        get a fresh pool, no further graphs are captured and the caller runs
        the chunk eagerly (returns None).

        ``empty_cache`` frees with ``hipFree``, which waits for ALL work on the
        device while holding the interpreter lock: behind an RCCL gather pending
        on a dead member it stalled the whole node process, heartbeats included,
        until the communicator timed out (8-rank RCCL rehearsal, worker failover
        with 4 / 8 chunks in flight).  ``trim_ok(need)`` (set by the node,
        ``RoundPlane.collectives_quiet``) says whether to trim now: always when no
        collective can be pending; while an RCCL epoch runs only when the
        cache's unused part exceeds ``trim_slack_bytes`` (``need``: node
        processes sharing one GPU) and none of the node's gathers is in flight.
        A trim that may not run now stays wanted (``maybe_trim``)."""
        before = len(r._graphs)
        try:
            out = fn()
        except (RuntimeError, torch.cuda.OutOfMemoryError) as e:   # includes AcceleratorError
            log.warning("graph capture failed (%s); eager forwards from now on", e)
            self.graphs_broken = True
            with self.lock:
                self._pool = torch.cuda.graph_pool_handle()
                for rr in self.runners.values():
                    rr.graph_pool = self._pool
            return None
        if len(r._graphs) > before:
            self._trim_wanted = True
            self.maybe_trim()
        return out

    def maybe_trim(self) -> None:
        """``empty_cache`` after new captures, when ``trim_ok(need)`` allows it
        (see ``_capture``); otherwise it stays wanted for a later call."""
        if not self._trim_wanted:
            return
        need = torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device) \
            > self.trim_slack_bytes
        if self.trim_ok is None or self.trim_ok(need):
            self._trim_wanted = False
            torch.cuda.empty_cache()

    def _forward(self, r, images, packed, slot: int = 0):
        """cls, prob of ``images`` on the private stream (caller holds run_lock);
        with ``packed`` the (class, prob bits) pairs are also written there.
        Launch slot ``slot`` replays its own graph (own static buffers)."""
        n = images.shape[0]
        if not self.closed and packed is None and (self._can_capture(r) or r.has_graph(n, slot=slot)):
            got = self._capture(r, lambda: r.capture(n, slot=slot))
            if got is not None:
                sin, replay = got
                sin.copy_(images)
                return replay()
        return r.forward(images.contiguous(), packed=packed)

    def _enter(self, images):
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=self.device)
        s = self.stream
        s.wait_stream(torch.cuda.current_stream(self.device))   # images were produced there
        images.record_stream(s)
        return s

    def submit(self, model, images, start, end):
        """Launch one chunk (copy-in, graph replay, pinned D2H) on a free slot
        and return at once; ``.result()`` waits for it and frees the slot.
        At most two chunks are in flight per executor."""
        r = self.runner(model)
        n = images.shape[0]
        with self._slot_cv:
            while all(self._slot_busy):
                self._slot_cv.wait()
            slot = self._next_slot if not self._slot_busy[self._next_slot] else self._next_slot ^ 1
            self._slot_busy[slot] = True
            self._next_slot = slot ^ 1
        try:
            with torch.cuda.device(self.device), self.run_lock:
                s = self._enter(images)
                with torch.cuda.stream(s):
                    cls, prob = self._forward(r, images, None, slot)
                    host = self._slots[slot]
                    if host is None or host.shape[0] < n:
                        host = self._slots[slot] = torch.empty(max(n, 1024), 2, dtype=torch.int32, pin_memory=True)
                    out = host[:n]
                    out[:, 0].copy_(cls, non_blocking=True)          # pinned D2H, no pageable bounce
                    out[:, 1].copy_(prob.view(torch.int32), non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(s)
        except BaseException:
            self._release(slot)
            raise
        return _HipPending(self, slot, ev, out, model, images)

    def rerun_exact(self, model, images):
        """(cls, prob) of ``images`` on the all-f32-MFMA kernels: the fallback
        for a chunk whose split forward left fp16's range."""
        r = self.runner(model)
        with torch.cuda.device(self.device), self.run_lock:
            s = self._enter(images)
            with torch.cuda.stream(s):
                z = r.logits_f32_exact(images.contiguous())
                cls, prob = r.ops.softmax_top1(z)
                res = (cls.cpu().numpy().astype(np.int32), prob.cpu().numpy().astype(np.float32))
        return res

    def _release(self, slot: int) -> None:
        with self._slot_cv:
            self._slot_busy[slot] = False
            self._slot_cv.notify_all()

    def run(self, model, images, start, end):
        return self.submit(model, images, start, end).result()

    def run_packed(self, model, images, packed):
        """Device-resident result path (collective rounds): write (class, prob
        bits) pairs of ``images`` into the int32 [>= n, 2] device tensor
        ``packed`` (the RCCL gather's send buffer) on the current stream's
        order; nothing comes back to the host and the host does not wait.
        Returns (start, end) events around the forward on the private stream:
        the chunk's own GPU time, read later once ``end`` has completed."""
        r = self.runner(model)
        n = images.shape[0]
        with torch.cuda.device(self.device), self.run_lock:
            s = self._enter(images)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            base = images._base
            # a view of a resident dataset (ResidentSource): the window graph reads
            # the images in place from a device-side start index -- no input copy
            # (SDFS shards and other views keep the static-input graph: a window
            # graph per shard would be captured inside the serving path)
            window = (base is not None and is_resident(base) and base.dim() == images.dim() and images.is_contiguous()
                      and base.is_contiguous() and base.dtype == images.dtype
                      and tuple(base.shape[1:]) == tuple(images.shape[1:]))
            with torch.cuda.stream(s):
                ev0.record(s)
                can_graph = self._can_capture(r)
                done = False
                if window and (can_graph or r.has_window(base, n, packed=packed)):
                    if can_graph and not r.has_graph(n, packed=packed):
                        # the static-input form for this slot as well, now (warm-up
                        # rounds): a later non-resident view (an SDFS shard) must not
                        # capture it inside a timed or serving round
                        self._capture(r, lambda: r.capture(n, packed=packed))
                    per = images[0].numel() * images.element_size()
                    got = self._capture(r, lambda: r.capture_window(base, n, packed=packed))
                    if got is not None:
                        start, replay = got
                        start.fill_((images.data_ptr() - base.data_ptr()) // per)
                        replay()
                        done = True
                elif can_graph or (not self.closed and r.has_graph(n, packed=packed)):
                    got = self._capture(r, lambda: r.capture(n, packed=packed))
                    if got is not None:
                        sin, replay = got
                        sin.copy_(images)
                        replay()
                        done = True
                if not done:
                    r.forward(images.contiguous(), packed=packed)
                ev1.record(s)
            torch.cuda.current_stream(self.device).wait_stream(s)
        return ev0, ev1


    def close(self) -> None:
        """Release the captured graphs (under the process-wide capture lock);
        a chunk still running afterwards takes the eager path."""
        self.closed = True
        with self.run_lock:
            # chunks launched by submit() may still be replaying their graphs:
            # drain the private stream before the graphs are destroyed
            if self.stream is not None:
                self.stream.synchronize()
        with self.lock:
            runners = list(self.runners.values())
        for r in runners:
            r.close()


def make_executor(kind: str, device=None, seed: int = 0, dtype: str = "fp32", fp32_impl: str = "split") -> Executor:
    kind = kind.lower()
    if kind == "auto":
        kind = "hip" if torch.cuda.is_available() else "torch"
    if kind == "hip":
        return HipExecutor(device or "cuda", seed=seed, dtype=dtype, fp32_impl=fp32_impl)
    if kind == "torch":
        return TorchExecutor(device or "cpu", seed=seed)
    if kind == "fake":
        return FakeExecutor()
    raise ValueError(f"unknown executor {kind!r}")
