"""Image data path: where a worker's chunk of images comes from.

The reference worker reads ``./<model>/test_<i>.JPEG`` from local disk, one
PIL image per forward, and overwrites non-RGB files in place
(alexnet_resnet.py:24, 48-54).  Here a chunk ``[start, end]``
is served as one uint8 tensor ``[n, 224, 224, 3]`` already resident on the
worker's device:

  * ``SyntheticSource``  deterministic per-index images (bit-identical on CPU
    numpy and on the GPU kernel ``ops.synth_images``), so any worker produces
    the same image ``i`` and results do not depend on placement;
  * ``SdfsSource``       images stored in SDFS as raw uint8 shards
    (``images/shard_<k>``, ``shard_images`` per shard).  A worker reads the
    shards covering its chunk from its own replica when it holds one (else
    from a replica over the control plane) and keeps them in an HBM cache, so
    each shard crosses PCIe once: ``HbmStager`` copies through a pinned host
    buffer with a non-blocking H2D on a dedicated side stream
    (hipMemcpyAsync), overlapping compute on the default stream.
"""
from __future__ import annotations

import os
import threading
from collections import OrderedDict

import numpy as np
import torch

HW = 224
IMG_BYTES = HW * HW * 3
GROUPS = IMG_BYTES // 8

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + _GOLD
        x = (x ^ (x >> np.uint64(30))) * _M1
        x = (x ^ (x >> np.uint64(27))) * _M2
        return x ^ (x >> np.uint64(31))


def synth_images_cpu(seed: int, start: int, n: int) -> np.ndarray:
    """uint8 [n, 224, 224, 3]; same bytes as the GPU kernel."""
    idx = (np.arange(n, dtype=np.uint64)[:, None] + np.uint64(start)) * np.uint64(GROUPS) + \
        np.arange(GROUPS, dtype=np.uint64)[None, :]
    h = _splitmix64((np.uint64(seed) << np.uint64(32)) ^ idx)
    return h.astype("<u8").view(np.uint8).reshape(n, HW, HW, 3)


class SyntheticSource:
    def __init__(self, seed: int, device: torch.device | str = "cpu"):
        self.seed = int(seed)
        self.device = torch.device(device)

    def get(self, start: int, end: int) -> torch.Tensor:
        n = end - start + 1
        if self.device.type == "cuda":
            from .. import ops

            with torch.cuda.device(self.device):       # the kernel runs on this device's current stream
                return ops.synth_images(self.seed, start, n, self.device)
        return torch.from_numpy(synth_images_cpu(self.seed, start, n))


_RESIDENT: dict = {}     # data_ptr -> weakref of the ResidentSource tensors (HipExecutor.run_packed)


def is_resident(t: torch.Tensor) -> bool:
    """``t`` is a ResidentSource dataset tensor: its views are read in place by
    window graphs (one graph per dataset, not per SDFS shard or request)."""
    r = _RESIDENT.get(t.data_ptr())
    return r is not None and r() is t


class ResidentSource:
    """The synthetic dataset resident in HBM, as the raw bench loop holds it
    ("dataset replicated in every GPU's HBM"): images [0, n) generated once
    (same bytes as SyntheticSource) into ONE tensor and served as views, so a
    round's chunk costs no generation and -- through the executor's window
    graph over that tensor (HipExecutor.run_packed) -- no input copy.
    Requests past n are generated per request (SyntheticSource)."""

    def __init__(self, seed: int, device: torch.device | str):
        self.seed = int(seed)
        self.device = torch.device(device)
        self.data: torch.Tensor | None = None
        self._fallback = SyntheticSource(seed, device)

    def make_resident(self, n: int) -> None:
        """Make images [0, n) resident (outside a timed region)."""
        if self.device.type != "cuda" or (self.data is not None and self.data.shape[0] >= n):
            return
        from .. import ops

        with torch.cuda.device(self.device):
            self.data = ops.synth_images(self.seed, 0, n, self.device)
            torch.cuda.current_stream(self.device).synchronize()
        import weakref

        _RESIDENT[self.data.data_ptr()] = weakref.ref(self.data)

    def get(self, start: int, end: int) -> torch.Tensor:
        d = self.data
        if d is not None and end < d.shape[0]:
            return d[start:end + 1]
        return self._fallback.get(start, end)


class HbmStager:
    """Host -> HBM staging through pinned memory on a side stream.

    Two pinned buffers in ping-pong: while the DMA engine copies piece k out of
    one buffer (hipMemcpyAsync on the side stream), the host fills piece k+1
    into the other; a buffer is reused only after the event of ITS last copy,
    so the host memcpy and the DMA overlap instead of alternating."""

    def __init__(self, device: torch.device, pinned_bytes: int = 64 << 20, nbuf: int = 2):
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(device=self.device) if self.gpu else None
        per = max(1 << 20, pinned_bytes // nbuf)
        self.pinned = [torch.empty(per, dtype=torch.uint8, pin_memory=self.gpu) for _ in range(nbuf)]
        self._done = [None] * nbuf        # event of the last copy out of each buffer
        self.lock = threading.Lock()
        self.bytes_staged = 0
        # optional GPU timeline: ("h2d", start event, end event, bytes) per stage() call
        # on the side stream (bench.py lines it up against the forwards' events)
        self.timeline: list | None = None
        self._readers = None              # preadv thread pool of stage_file (lazy)
        self.native_read_s = 0.0          # native stager: time in pread / waiting for the DMA engine
        self.native_wait_s = 0.0

    READ_THREADS = 8

    def _native(self):
        """The extension's GIL-free file stager (None: the Python preadv path)."""
        if not self.gpu or os.environ.get("IDUNNO_PY_STAGING") == "1":
            return None
        try:
            from .. import ops

            return getattr(ops.load(), "stage_file_native", None)
        except Exception:  # noqa: BLE001  (no extension: the Python path)
            return None

    def stage_file(self, path: str, shape: tuple) -> torch.Tensor:
        """``_stage_file`` with the current stream ordered after the copy."""
        t, ev = self._stage_file(path, shape)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return t

    def _stage_file(self, path: str, shape: tuple):
        """Stage a file's bytes into a new device tensor of ``shape`` (uint8)
        without a host copy of the file: each piece is read with ``os.preadv``
        by up to READ_THREADS threads straight into a pinned ping-pong buffer (the
        reads release the GIL), then DMA'd on the side stream while the next
        piece is read into the other buffer.  A bytes object of a large file
        costs fresh page faults on every read (~1.5 GB/s on these hosts); the
        pinned buffers are faulted in once.  Returns (tensor, event of its last
        copy); the tensor is allocated on the side stream (hand-outs to other
        streams call ``record_stream``, see SdfsSource._shard)."""
        nbytes = int(np.prod(shape))
        fd = os.open(path, os.O_RDONLY)
        try:
            if os.fstat(fd).st_size < nbytes:
                raise ValueError(f"{path}: {os.fstat(fd).st_size} bytes, need {nbytes}")
            if not self.gpu:
                buf = np.empty(nbytes, np.uint8)
                self._pread(fd, memoryview(buf), 0)
                self.bytes_staged += nbytes
                return torch.from_numpy(buf).view(*shape), None
            with torch.cuda.stream(self.stream):
                out = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            step = self.pinned[0].numel()
            nb = len(self.pinned)
            native = self._native()
            with self.lock:
                ev = None
                tl = self.timeline
                if tl is not None:
                    ev0 = torch.cuda.Event(enable_timing=True)
                    ev0.record(self.stream)
                if native is not None:
                    # the whole file with the GIL released (csrc/runtime/staging.cpp); it
                    # returns once the pinned buffers are free again
                    for b in range(nb):
                        if self._done[b] is not None:
                            self._done[b].synchronize()
                            self._done[b] = None
                    tr, tw, tt = native(path, out, self.pinned, self.stream.cuda_stream, self.READ_THREADS)
                    self.native_read_s += tr
                    self.native_wait_s += tw + tt
                    with torch.cuda.stream(self.stream):
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                    nbytes_left = 0
                else:
                    nbytes_left = nbytes
                for i, off in enumerate(range(0, nbytes_left, step)):
                    b = i % nb
                    n = min(step, nbytes - off)
                    if self._done[b] is not None:
                        self._done[b].synchronize()
                    self._pread(fd, memoryview(self.pinned[b].numpy())[:n], off)
                    with torch.cuda.stream(self.stream):
                        out[off:off + n].copy_(self.pinned[b][:n], non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                    self._done[b] = ev
                if tl is not None:
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record(self.stream)
                    tl.append(("h2d", ev0, ev1, nbytes))
                self.bytes_staged += nbytes
        finally:
            os.close(fd)
        return out.view(*shape), ev

    def _pread(self, fd: int, dst: memoryview, off: int) -> None:
        """Fill ``dst`` from file offset ``off`` with parallel preadv calls."""
        n = len(dst)
        nt = max(1, min(self.READ_THREADS, n >> 22))          # >= 4 MiB per thread
        part = -(-n // nt)

        def work(i):
            mv, pos = dst[i * part:min(n, (i + 1) * part)], off + i * part
            while len(mv):
                k = os.preadv(fd, [mv], pos)
                if k <= 0:
                    raise EOFError(f"short read at {pos}")
                mv, pos = mv[k:], pos + k
        if nt == 1:
            work(0)
            return
        if self._readers is None:
            from concurrent.futures import ThreadPoolExecutor

            self._readers = ThreadPoolExecutor(max_workers=self.READ_THREADS, thread_name_prefix="stage-read")
        futs = [self._readers.submit(work, i) for i in range(nt)]
        errs = [f.exception() for f in futs]        # every read has ended before the fd can close
        for e in errs:
            if e is not None:
                raise e

    def stage(self, data: bytes | np.ndarray, shape: tuple) -> torch.Tensor:
        """Copy host bytes to a new device tensor of ``shape`` (uint8).  The
        current stream is made to wait for the copy; nothing blocks the host
        beyond the ping-pong buffer reuse."""
        t, ev = self._stage(data, shape)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return t

    def _stage(self, data, shape: tuple):
        """``stage`` without the current-stream wait: (tensor, event of its
        last copy), the tensor allocated on the side stream."""
        src = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) \
            else np.ascontiguousarray(data).reshape(-1).view(np.uint8)
        if not self.gpu:
            self.bytes_staged += src.size
            return torch.from_numpy(src.copy()).view(*shape), None
        with torch.cuda.stream(self.stream):
            out = torch.empty(src.size, dtype=torch.uint8, device=self.device)
        step = self.pinned[0].numel()
        nb = len(self.pinned)
        with self.lock:
            ev = None
            tl = self.timeline
            if tl is not None:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record(self.stream)
            for i, off in enumerate(range(0, src.size, step)):
                b = i % nb
                n = min(step, src.size - off)
                if self._done[b] is not None:
                    self._done[b].synchronize()     # the DMA that last read buffer b has finished
                self.pinned[b][:n].numpy()[:] = src[off:off + n]
                with torch.cuda.stream(self.stream):
                    out[off:off + n].copy_(self.pinned[b][:n], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                self._done[b] = ev
            if tl is not None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record(self.stream)
                tl.append(("h2d", ev0, ev1, src.size))
            self.bytes_staged += src.size
        return out.view(*shape), ev


def shard_name(k: int) -> str:
    return f"images/shard_{k:05d}"


class SdfsSource:
    """Images from SDFS shards, cached in HBM (LRU by bytes).

    A shard another node already holds in HBM is copied GPU-to-GPU from that
    node (SDFS FETCH_HBM + runtime/ipc.py) instead of being read from a
    replica over TCP and staged host->HBM; every shard this node caches is
    announced to the SDFS master so peers can do the same (``peer_copy``)."""

    def __init__(self, sdfs, device, shard_images: int = 500, cache_bytes: int = 32 << 30, peer_copy: bool = True,
                 readahead: int = 1, stage_streams: int = 1):
        self.sdfs = sdfs
        self.device = torch.device(device)
        self.S = int(shard_images)
        # shards stage on `stage_streams` side streams at once (one stager, pinned pair and
        # background worker each).  Two measured no faster than one on the cold SDFS pass
        # (0.70 vs 0.74 cold/warm): the copies themselves run at ~45 GB/s beside the
        # forwards (tools/overlap_probe.py under rocprofv3); the host reads set the pace
        self.nstage = max(1, int(stage_streams)) if self.device.type == "cuda" else 1
        self.stagers = [HbmStager(self.device) for _ in range(self.nstage)]
        self.stager = self.stagers[0]
        self.cache: OrderedDict[int, torch.Tensor] = OrderedDict()
        self.ver: dict[int, int] = {}             # SDFS version of each cached shard
        self.cache_bytes = cache_bytes
        self.lock = threading.Lock()
        self.fetches = 0
        self.peer_fetches = 0
        self.peer_copy = peer_copy and self.device.type == "cuda"
        # sequential readahead: a request for shard k starts shard k+1 .. k+readahead on
        # a background thread, so its SDFS read and H2D copy (side stream) run while the
        # current chunk computes instead of in front of the next one
        self.readahead = int(readahead)
        self.max_queued = max(2, 2 * self.readahead)   # background fetches queued or running at most
        self._inflight: dict[int, object] = {}     # shard -> Future of a background fetch
        self._ready: dict[int, object] = {}        # shard -> event of its last H2D copy (side stream)
        self._rec: set = set()                    # (shard, stream) pairs already record_stream'ed
        self._ahead: set = set()                  # shards a background fetch put in the cache
        self._absent: set = set()                 # shards a readahead found missing (past the dataset's end)
        self._pool = None
        self.readahead_hits = 0
        self.local_reads = 0                      # shards streamed from this node's own replica file
        self.tracer = None                        # optional utils.tracing.Tracer: "sdfs.fetch" spans
        if self.device.type == "cuda":
            sdfs.hbm_provider = self.export_shard

    def cached(self, start: int, end: int) -> bool:
        """All shards of [start, end] already in HBM (get() will not fetch)."""
        with self.lock:
            return all(k in self.cache for k in range(start // self.S, end // self.S + 1))

    def export_shard(self, name: str, consumer_pid: int | None = None, ver: int | None = None):
        """IPC export of a cached shard (SDFS FETCH_HBM), or None -- also when
        the cached copy is not of the requested version ``ver``."""
        from .ipc import export_tensor

        with self.lock:
            k = next((k for k in self.cache if shard_name(k) == name), None)
            t = self.cache.get(k) if k is not None else None
            if t is not None and ver is not None and self.ver.get(k) != int(ver):
                t = None
            ev = self._ready.get(k) if t is not None else None
        if t is None:
            return None
        if ev is not None:
            ev.synchronize()                                      # its staged bytes have landed
        else:
            torch.cuda.current_stream(self.device).synchronize()
        return export_tensor(t, consumer_pid)

    def _prefetch(self, k: int, requested: bool = False) -> None:
        """Start fetching shard k in the background unless cached or in flight.
        ``stage_streams`` workers, FIFO, so shards start staging in request order.  Speculative
        readahead (past a request) is bounded to ``max_queued`` background
        fetches; a shard an announced chunk needs (``requested``) always queues."""
        with self.lock:
            if k in self.cache or k in self._inflight or k in self._absent:
                return
            if not requested and len(self._inflight) >= self.max_queued:
                return
            if self._pool is None:
                from concurrent.futures import ThreadPoolExecutor

                self._pool = ThreadPoolExecutor(max_workers=self.nstage, thread_name_prefix="sdfs-readahead")
            dev = self.device

            def run():
                import contextlib

                ctx = torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext()
                try:
                    with ctx:
                        t = self._fetch(k)
                    with self.lock:
                        self._ahead.add(k)
                    return t
                except KeyError:
                    with self.lock:
                        self._absent.add(k)              # not asked again by readahead
                    raise
                finally:
                    with self.lock:
                        self._inflight.pop(k, None)
            self._inflight[k] = self._pool.submit(run)

    def prefetch(self, start: int, end: int) -> None:
        """Start staging every shard of images [start, end] in the background
        (in request order, behind shards already queued)."""
        for k in range(start // self.S, end // self.S + 1):
            self._prefetch(k, requested=True)

    def _shard(self, k: int) -> torch.Tensor:
        with self.lock:
            t = self.cache.get(k)
            if t is not None:
                self.cache.move_to_end(k)
            fut = self._inflight.get(k) if t is None else None
        if t is None and fut is not None:
            try:
                t = fut.result()
            except Exception:  # noqa: BLE001  (fetch again below; a missing shard raises there)
                t = None
        if t is None:
            t = self._fetch(k)
        return self._hand_out(k, t)

    def _hand_out(self, k: int, t: torch.Tensor) -> torch.Tensor:
        """Order the caller's current stream after shard k's own H2D copy (its
        event, not the whole side stream, which may hold later readahead), and
        record that stream on the tensor so the allocator keeps the block until
        the consumer's work is done if the shard is evicted."""
        with self.lock:
            if k in self._ahead:
                self._ahead.discard(k)
                self.readahead_hits += 1
            ev = self._ready.get(k)
        if self.device.type == "cuda":
            cs = torch.cuda.current_stream(self.device)
            if ev is not None:
                cs.wait_event(ev)
            key = (k, cs.cuda_stream)
            with self.lock:
                fresh = key not in self._rec and self.cache.get(k) is t
                if fresh:
                    self._rec.add(key)
            if fresh:
                t.record_stream(cs)
            elif self.cache.get(k) is not t:
                t.record_stream(cs)           # not the cached tensor (evicted meanwhile): always
        return t

    def _fetch(self, k: int) -> torch.Tensor:
        if self.tracer is None:
            return self._fetch_body(k)
        with self.tracer.span("sdfs.fetch", shard=k):
            return self._fetch_body(k)

    def _fetch_body(self, k: int) -> torch.Tensor:
        with self.lock:
            t = self.cache.get(k)
            if t is not None:
                return t
        name = shard_name(k)
        got = self.sdfs.fetch_hbm(name, self.device) if self.peer_copy else None
        ev = None
        if got is not None:
            t, ver = got
            self.peer_fetches += 1
        else:
            # this node's own replica streams from its file into the pinned buffers;
            # another node's replica comes over the transport as bytes
            loc = self.sdfs.local_file(name) if hasattr(self.sdfs, "local_file") else None
            if loc is not None:
                path, ver = loc
                try:
                    n = os.path.getsize(path) // IMG_BYTES
                    t, ev = self.stagers[k % self.nstage]._stage_file(path, (n, HW, HW, 3))
                    self.local_reads += 1
                except OSError:                   # replaced by a newer version meanwhile
                    loc = None
            if loc is None:
                got = self.sdfs.get_bytes_ver(name)
                if got is None:
                    raise KeyError(f"missing SDFS shard {name}")
                data, ver = got
                n = len(data) // IMG_BYTES
                t, ev = self.stagers[k % self.nstage]._stage(data, (n, HW, HW, 3))
        dropped = []
        with self.lock:
            held = self.cache.get(k)
            if held is not None:
                # another fetch of k (round thread vs background readahead) filled the
                # cache first: keep that tensor -- consumers may already hold it and
                # record_stream'ed it -- and drop this duplicate (its copy is ordered
                # on the stager's stream, which is the stream its block returns to)
                return held
            self.fetches += 1
            self._rec = {x for x in self._rec if x[0] != k}
            self.cache[k] = t
            self.ver[k] = ver
            self._ready[k] = ev
            tot = sum(v.numel() for v in self.cache.values())
            while tot > self.cache_bytes and len(self.cache) > 1:
                ko, old = self.cache.popitem(last=False)
                self.ver.pop(ko, None)
                self._ready.pop(ko, None)
                self._ahead.discard(ko)
                self._rec = {x for x in self._rec if x[0] != ko}
                tot -= old.numel()
                dropped.append(ko)
        if self.device.type == "cuda":
            self.sdfs.announce_hbm(name, ver=ver)
            for ko in dropped:
                self.sdfs.announce_hbm(shard_name(ko), held=False)
        return t

    def get(self, start: int, end: int) -> torch.Tensor:
        parts = []
        i = start
        last = end // self.S
        while i <= end:
            k = i // self.S
            sh = self._shard(k)
            lo = i - k * self.S
            hi = min(end - k * self.S, sh.shape[0] - 1)
            if hi < lo:
                raise KeyError(f"image {i} beyond shard {k}")
            parts.append(sh[lo:hi + 1])
            i = k * self.S + hi + 1
        # readahead once this request's shards are in hand: a background fetch that
        # took the stager first would put a whole shard in front of the one needed now
        for r in range(1, self.readahead + 1):
            self._prefetch(last + r)
        if len(parts) == 1:
            return parts[0]
        # joined with async copies, not torch.cat: the first cat of a process loads
        # its kernel's code object, which waited for the in-flight H2D staging to
        # drain and held the round thread 14-25 ms in the cold SDFS pass
        # (profiles/r5_sdfs_trace_before.json, tools/alloc_probe.py)
        out = torch.empty((sum(p.shape[0] for p in parts), *parts[0].shape[1:]), dtype=parts[0].dtype,
                          device=parts[0].device)
        i = 0
        for p in parts:
            out[i:i + p.shape[0]].copy_(p, non_blocking=True)
            i += p.shape[0]
        return out


def load_image_u8(data: bytes, resize: int = 256, crop: int = 224) -> np.ndarray:
    """Decode one image and apply the reference's Resize(256) + CenterCrop(224)
    (alexnet_resnet.py:50-59) with PIL, returning uint8 [crop, crop, 3].
    Non-RGB images are converted in memory; the source file is never
    rewritten (the reference overwrites it on disk)."""
    import io

    from PIL import Image

    im = Image.open(io.BytesIO(data))
    if im.mode != "RGB":
        im = im.convert("RGB")
    w, h = im.size
    if w <= h:
        nw, nh = resize, int(resize * h / w)
    else:
        nh, nw = resize, int(resize * w / h)
    im = im.resize((nw, nh), Image.BILINEAR)
    left, top = int(round((nw - crop) / 2.0)), int(round((nh - crop) / 2.0))
    im = im.crop((left, top, left + crop, top + crop))
    return np.asarray(im, dtype=np.uint8)


class JpegSource:
    """Real image files ``test_<i>.JPEG`` (the reference's dataset naming,
    alexnet_resnet.py:49) read from a local directory or from SDFS, decoded and
    resized on host threads, staged to HBM in one copy per chunk.  A missing
    image becomes an all-zero image and is reported in ``missing``."""

    def __init__(self, device, root: str | None = None, sdfs=None, prefix: str = "", workers: int = 8):
        from concurrent.futures import ThreadPoolExecutor

        self.device = torch.device(device)
        self.root, self.sdfs, self.prefix = root, sdfs, prefix
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.stager = HbmStager(self.device)
        self.missing: list[int] = []

    def _read(self, i: int) -> bytes | None:
        name = f"{self.prefix}test_{i}.JPEG"
        if self.sdfs is not None:
            return self.sdfs.get_bytes(name)
        import os

        p = os.path.join(self.root, name)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            return f.read()

    def _one(self, i: int) -> np.ndarray:
        data = self._read(i)
        if data is None:
            self.missing.append(i)
            return np.zeros((HW, HW, 3), np.uint8)
        return load_image_u8(data)

    def cached(self, start: int, end: int) -> bool:
        return False                      # every chunk decodes on host threads

    def get(self, start: int, end: int) -> torch.Tensor:
        arr = np.stack(list(self.pool.map(self._one, range(start, end + 1))))
        return self.stager.stage(arr, arr.shape)


def put_synthetic_dataset(sdfs, n_images: int, seed: int, shard_images: int = 500) -> int:
    """Upload a deterministic synthetic dataset into SDFS as uint8 shards."""
    k = 0
    for s in range(0, n_images, shard_images):
        n = min(shard_images, n_images - s)
        sdfs.put_bytes(synth_images_cpu(seed, s, n).tobytes(), shard_name(k))
        k += 1
    return k
