"""One-process-per-GPU data plane over RCCL (torch.distributed "nccl" == RCCL
on ROCm; xGMI between the 8 MI355X of a node).

Replaces the reference's per-chunk TCP messages on the hot path
(SURVEY.md §2.5):
  * M9  INFERENCE chunk dispatch (coordinator -> workers)   -> ``dispatch``:
        one broadcast of a tiny int64 descriptor table [world, 4]
        (model_id, query_id, start, end) per query round;
  * M11 RESULT broadcast of stringified tuples to all 10 hosts -> ``gather``:
        one RCCL gather of packed top-1 results (int32 class + fp32 prob,
        8 B/image, 3.2 KB for a 400-image chunk) to the coordinator rank
        (and, optionally, a second one to the standby rank).
  * M9  data variant -> ``scatter`` / ``scatter_async``: the coordinator
        holds a query's images in HBM and sends every rank its chunk with one
        grouped point-to-point send per peer, so the 7 xGMI links of the root
        carry the shards concurrently (60 MB per 400-image chunk); bench.py
        measures it double-buffered against compute (``images_per_s_scatter``).
In steady state images do not cross the fabric at all: every rank stages its
own shard host->HBM (``idunno.runtime.data.HbmStager`` / ``SdfsSource``) and
``scatter`` is used only when the images live on the coordinator.

On CPU (tests) the same code runs over gloo.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

NO_WORK = -1


@dataclass
class Env:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def distributed(self) -> bool:
        return self.world > 1


def init_from_env(backend: str | None = None, timeout_s: float = 300.0, cpu: bool = False) -> Env:
    """Initialise the default process group from torchrun-style env vars
    (``cpu``: stay off the GPU even where one exists -- gloo dry runs)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    gpu = not cpu and torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    backend = backend or ("nccl" if gpu else "gloo")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        from datetime import timedelta

        kw = {}
        if backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=timedelta(seconds=timeout_s), **kw)
    return Env(rank, world, local, device, backend)


class QueryPlane:
    """Collective dispatch / gather between the coordinator rank and workers."""

    def __init__(self, env: Env, coordinator: int = 0, max_chunk: int = 512, group=None, nbuf: int = 1):
        self.env = env
        self.coord = coordinator
        self.max_chunk = max_chunk
        self.group = group
        self.nbuf = nbuf
        dev = env.device
        # nbuf slots of descriptor table / send buffer / gathered round: with 2, round
        # q+1's descriptor broadcast and round q's gather run on the collective stream
        # while the other slot's forward computes (post_dispatch / post_gather)
        self._descs = torch.full((nbuf, env.world, 4), NO_WORK, dtype=torch.int64, device=dev)
        self._desc = self._descs[0]
        # one contiguous [world, max_chunk, 2] buffer per slot on the coordinator; the
        # per-rank gather outputs are views of it, so the whole round's results
        # come to the host with ONE device->host copy (``gathered_all``)
        coord = env.rank == coordinator
        self._gathered_slots = [torch.zeros(env.world, max_chunk, 2, dtype=torch.int32, device=dev)
                                for _ in range(nbuf)] if coord else None
        self.gathered_all = self._gathered_slots[0] if coord else None
        self._gathered = list(self.gathered_all.unbind(0)) if coord else None
        # send buffers; a single rank's results are already in place (no copy)
        if env.world == 1:
            self._packs = [g[0] for g in self._gathered_slots]
        else:
            self._packs = [torch.zeros(max_chunk, 2, dtype=torch.int32, device=dev) for _ in range(nbuf)]
        self._pack = self._packs[0]
        self._desc_host = None
        # scatter buckets: each peer's shard goes as SCATTER_BUCKET_BYTES pieces posted
        # round-robin over the peers in one group, so all 7 xGMI links of the root
        # carry data from the first piece on and a peer's receive completes piecewise
        self.scatter_bucket_bytes = self.SCATTER_BUCKET_BYTES

    SCATTER_BUCKET_BYTES = 4 << 20

    # -- M9 ---------------------------------------------------------------------
    def dispatch(self, table: list[tuple[int, int, int, int]] | None) -> tuple[int, int, int, int]:
        """Coordinator passes one (model_id, qid, start, end) row per rank
        (end = -1 for an idle rank); every rank gets its own row back."""
        if self.env.rank == self.coord:
            assert table is not None and len(table) == self.env.world
            for r, row in enumerate(table):
                if row[3] != NO_WORK and row[3] - row[2] + 1 > self.max_chunk:
                    raise ValueError(f"chunk {row} larger than max_chunk={self.max_chunk}")
            self._desc.copy_(torch.tensor(table, dtype=torch.int64), non_blocking=True)
        if self.env.distributed:
            dist.broadcast(self._desc, src=self.coord, group=self.group)
        row = self._desc[self.env.rank].tolist()
        return tuple(int(v) for v in row)

    def dispatch_async(self, table: list[tuple[int, int, int, int]] | None):
        """Start the descriptor broadcast; returns the collective's Work (None
        on a single rank).  The row is in ``self._desc`` once it completed."""
        if self.env.rank == self.coord:
            assert table is not None and len(table) == self.env.world
            for row in table:
                if row[3] != NO_WORK and row[3] - row[2] + 1 > self.max_chunk:
                    raise ValueError(f"chunk {row} larger than max_chunk={self.max_chunk}")
            self._desc.copy_(torch.tensor(table, dtype=torch.int64), non_blocking=True)
        if not self.env.distributed:
            return None
        return dist.broadcast(self._desc, src=self.coord, group=self.group, async_op=True)

    def my_row(self) -> tuple[int, int, int, int]:
        return tuple(int(v) for v in self._desc[self.env.rank].tolist())

    def gather_async(self):
        """Start the gather of the send buffer to the coordinator (Work or None)."""
        if not self.env.distributed:
            return None
        if self.env.rank == self.coord:
            return dist.gather(self._pack, self._gathered, dst=self.coord, group=self.group, async_op=True)
        return dist.gather(self._pack, None, dst=self.coord, group=self.group, async_op=True)

    # -- double-buffered rounds (bench.py's raw loop at N > 1) -------------------------
    def row_start_slot(self, slot: int) -> torch.Tensor:
        return self._descs[slot, self.env.rank, 2:3]

    def send_slot(self, slot: int) -> torch.Tensor:
        return self._packs[slot]

    def gathered_slot(self, slot: int) -> torch.Tensor | None:
        return self._gathered_slots[slot] if self._gathered_slots is not None else None

    def post_dispatch(self, table, slot: int, hslot: int):
        """Descriptor table of a round into slot ``slot`` (coordinator: staged
        through pinned host buffer ``hslot % 4``) and its broadcast, without
        waiting: returns the Work (None on one rank).  Post it BEFORE queuing
        the forward that overlaps it and after the forward that last read the
        slot (the collective stream waits for the work queued before it)."""
        if self._desc_host is None:
            pin = self.env.device.type == "cuda"
            self._desc_host = [torch.full((self.env.world, 4), NO_WORK, dtype=torch.int64, pin_memory=pin)
                               for _ in range(4)]
        d = self._descs[slot]
        if self.env.rank == self.coord:
            assert table is not None and len(table) == self.env.world
            h = self._desc_host[hslot % 4]
            h.copy_(torch.tensor(table, dtype=torch.int64))
            d.copy_(h, non_blocking=True)
        if not self.env.distributed:
            return None
        return dist.broadcast(d, src=self.coord, group=self.group, async_op=True)

    def post_gather(self, slot: int):
        """Gather of slot ``slot``'s send buffer into its gathered round
        (coordinator), without waiting; None on one rank."""
        if not self.env.distributed:
            return None
        outs = list(self._gathered_slots[slot].unbind(0)) if self.env.rank == self.coord else None
        return dist.gather(self._packs[slot], outs, dst=self.coord, group=self.group, async_op=True)

    @staticmethod
    def wait_work(work) -> None:
        """The current stream (RCCL) waits for ``work``; the host does not."""
        if work is not None:
            work.wait()

    def dispatch_device(self, table: list[tuple[int, int, int, int]] | None, slot: int = 0) -> torch.Tensor:
        """Asynchronous dispatch: no host synchronisation anywhere.

        The coordinator stages the table in pinned host memory (``slot`` picks
        one of two buffers so a table is never overwritten while its copy is
        in flight), copies it to the device and broadcasts it; every rank gets
        back a *device* view of its own row, which the forward graph consumes
        directly (e.g. as the shard window start)."""
        if self._desc_host is None:
            pin = self.env.device.type == "cuda"
            self._desc_host = [torch.full((self.env.world, 4), NO_WORK, dtype=torch.int64, pin_memory=pin)
                               for _ in range(4)]
        if self.env.rank == self.coord:
            assert table is not None and len(table) == self.env.world
            h = self._desc_host[slot % 2]
            h.copy_(torch.tensor(table, dtype=torch.int64))
            self._desc.copy_(h, non_blocking=True)
        if self.env.distributed:
            dist.broadcast(self._desc, src=self.coord, group=self.group)
        return self._desc[self.env.rank]

    def scatter(self, images: torch.Tensor | None, table, row, img_shape=(224, 224, 3)):
        """Send every rank its chunk of the coordinator's images.

        ``images`` (coordinator only) holds the query's images ``[B, *img_shape]``
        with row 0 = the smallest start in ``table``; ``row`` is this rank's
        descriptor from ``dispatch``.  Returns this rank's ``[n, *img_shape]``
        images (a view on the coordinator, a reused receive buffer elsewhere) or
        None for an idle rank."""
        s, e = int(row[2]), int(row[3])
        n = 0 if e == NO_WORK else e - s + 1
        if self.env.rank == self.coord:
            base = min(r[2] for r in table if r[3] != NO_WORK)
            src = images.contiguous()
            shards = {peer: (r[2] - base, r[3] - base) for peer, r in enumerate(table)
                      if peer != self.coord and r[3] != NO_WORK}
            ops = self._send_ops(src, shards)
            if ops and self.env.distributed:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            return images[s - base:e + 1 - base] if n else None
        if n == 0:
            return None
        if getattr(self, "_recv", None) is None or tuple(self._recv.shape[1:]) != tuple(img_shape):
            self._recv = torch.empty((self.max_chunk, *img_shape), dtype=torch.uint8, device=self.env.device)
        buf = self._recv[:n]
        for req in dist.batch_isend_irecv(self._recv_ops(buf)):
            req.wait()
        return buf

    def _bucket_rows(self, row_bytes: int) -> int:
        b = int(self.scatter_bucket_bytes)
        return max(1, b // max(1, row_bytes)) if b > 0 else 1 << 62

    def _send_ops(self, images: torch.Tensor, shards: dict) -> list:
        """Root: isend ops of every peer's rows [a, b] of ``images`` in buckets
        of ``scatter_bucket_bytes``, interleaved round-robin over the peers
        (bucket 0 of every peer, then bucket 1, ...).  P2P between one pair of
        ranks matches in posting order, so ``_recv_ops`` mirrors the split."""
        step = self._bucket_rows(images[0].numel() * images.element_size()) if images.numel() else 1
        pieces = {p: [(i, min(i + step - 1, b)) for i in range(a, b + 1, step)] for p, (a, b) in shards.items()}
        ops = []
        for k in range(max((len(v) for v in pieces.values()), default=0)):
            for p, v in pieces.items():
                if k < len(v):
                    ops.append(dist.P2POp(dist.isend, images[v[k][0]:v[k][1] + 1], p, self.group))
        return ops

    def _recv_ops(self, buf: torch.Tensor) -> list:
        """Member: irecv ops of its shard ``buf`` in the root's bucket split."""
        step = self._bucket_rows(buf[0].numel() * buf.element_size()) if buf.numel() else 1
        return [dist.P2POp(dist.irecv, buf[i:i + step], self.coord, self.group) for i in range(0, buf.shape[0], step)]

    def scatter_async(self, images: torch.Tensor | None, chunks, out: torch.Tensor) -> list:
        """Non-blocking fixed-size scatter into ``out`` (every rank's receive
        buffer, [n, ...]): the coordinator sends rank r the rows
        ``images[chunks[r][0]:chunks[r][1] + 1]`` (one group of P2P ops, every
        peer's shard in ``scatter_bucket_bytes`` buckets posted round-robin over
        the peers: the root's 7 xGMI links carry the shards concurrently) and
        copies its own chunk into ``out``.  Returns the requests; ``wait_scatter`` makes
        the CURRENT stream wait for them (RCCL) -- the host does not block.

        Ordering on RCCL: the communication stream waits for the work queued
        on the current stream when the ops are posted, so post a buffer's
        next scatter BEFORE queuing the compute that overlaps it and AFTER the
        compute that last read that buffer."""
        if self.env.rank == self.coord:
            s0, e0 = chunks[self.coord]
            out[: e0 - s0 + 1].copy_(images[s0:e0 + 1], non_blocking=True)
            ops = self._send_ops(images, {peer: (s, e) for peer, (s, e) in enumerate(chunks) if peer != self.coord})
        else:
            s, e = chunks[self.env.rank]
            ops = self._recv_ops(out[: e - s + 1])
        if not ops or not self.env.distributed:
            return []
        return dist.batch_isend_irecv(ops)

    @staticmethod
    def wait_scatter(reqs: list) -> None:
        for r in reqs:
            r.wait()

    # -- M11 --------------------------------------------------------------------
    @property
    def send_buffer(self) -> torch.Tensor:
        """[max_chunk, 2] int32 (class, prob bits): a forward that writes its
        results here directly (``HipRunner.capture_window(packed=...)``)
        calls ``gather(None, None)``."""
        return self._pack

    def row_start(self) -> torch.Tensor:
        """Device view of this rank's descriptor start field (int64 [1]): the
        forward graph reads its shard window start from it in place."""
        return self._desc[self.env.rank, 2:3]

    def pack(self, cls: torch.Tensor, prob: torch.Tensor) -> torch.Tensor:
        n = cls.numel()
        self._pack[:n, 0].copy_(cls.view(-1).to(torch.int32))
        self._pack[:n, 1].copy_(prob.view(-1).float().view(torch.int32))
        return self._pack

    def gather(self, cls: torch.Tensor | None, prob: torch.Tensor | None):
        """Gather packed top-1 results to the coordinator.  Returns, on the
        coordinator, a list (per rank) of int32 [max_chunk, 2] device tensors."""
        if cls is not None:
            self.pack(cls, prob)
        if not self.env.distributed:
            return self._gathered            # _pack IS _gathered[0]
        if self.env.rank == self.coord:
            dist.gather(self._pack, self._gathered, dst=self.coord, group=self.group)
            return self._gathered
        dist.gather(self._pack, None, dst=self.coord, group=self.group)
        return None


def unpack(packed: torch.Tensor, n: int) -> tuple[torch.Tensor, torch.Tensor]:
    """(cls int32 [n], prob fp32 [n]) from a packed [*, 2] int32 tensor (any device)."""
    p = packed[:n]
    return p[:, 0].clone(), p[:, 1].clone().view(torch.float32)
