"""RCCL data-plane logic (dispatch broadcast + top-1 gather) exercised over
gloo with world_size 2 / 3 on the CPU — the same code bench.py runs over RCCL."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from idunno.parallel.dataplane import NO_WORK, QueryPlane, init_from_env, unpack
    from idunno.runtime.executor import FakeExecutor
    from idunno.runtime.scheduler import split_range

    env = init_from_env(backend="gloo")
    plane = QueryPlane(env, coordinator=0, max_chunk=64)
    ex = FakeExecutor()
    out = {}
    for step in range(3):
        table = None
        if env.rank == 0:
            chunks = split_range(step * 100, step * 100 + 99, world)
            table = [(1, step, s, e) for s, e in chunks]
            table += [(1, step, 0, NO_WORK)] * (world - len(table))
        if step % 2:
            mid, qid, s, e = plane.dispatch(table)
        else:                                   # the asynchronous (device-row) variant bench.py uses
            mid, qid, s, e = (int(v) for v in plane.dispatch_device(table, slot=step).tolist())
        cls, prob = ex.run("resnet18", None, s, e)
        g = plane.gather(torch.from_numpy(cls), torch.from_numpy(prob))
        if env.rank == 0:
            for r in range(world):
                c, p = unpack(g[r], table[r][3] - table[r][2] + 1)
                for i, (cc, pp) in enumerate(zip(c.tolist(), p.tolist())):
                    out[table[r][2] + i] = (cc, pp)
    if env.rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_dispatch_gather_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert sorted(out) == list(range(300))
    for i, (c, p) in out.items():
        assert c == (i * 7919 + 13) % 1000 and abs(p - 0.5) < 1e-7


def _scatter_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist

    from idunno.parallel.dataplane import NO_WORK, QueryPlane, init_from_env
    from idunno.runtime.data import synth_images_cpu
    from idunno.runtime.scheduler import split_range

    env = init_from_env(backend="gloo")
    plane = QueryPlane(env, coordinator=0, max_chunk=16)
    ok = True
    for step, (s0, e0) in enumerate([(100, 129), (7, 8)]):
        table = imgs = None
        if env.rank == 0:
            chunks = split_range(s0, e0, world)
            table = [(1, step, s, e) for s, e in chunks] + [(1, step, 0, NO_WORK)] * (world - len(chunks))
            imgs = torch.from_numpy(synth_images_cpu(5, s0, e0 - s0 + 1))
        row = plane.dispatch(table)
        got = plane.scatter(imgs, table, row)
        if row[3] == NO_WORK:
            ok &= got is None
        else:
            ok &= np.array_equal(got.numpy(), synth_images_cpu(5, row[2], row[3] - row[2] + 1))
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_scatter_images_over_gloo():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res == {r: True for r in range(world)}


def _scatter_async_worker(rank, world, port, q):
    """bench.py's scatter rounds: fixed-size chunks into two receive buffers,
    round r+1 posted before round r is consumed (double buffering)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist

    from idunno.parallel.dataplane import QueryPlane, init_from_env
    from idunno.runtime.data import synth_images_cpu
    from idunno.runtime.scheduler import split_range

    env = init_from_env(backend="gloo")
    plane = QueryPlane(env, coordinator=0, max_chunk=6)
    B, D = 6, 60
    src = torch.from_numpy(synth_images_cpu(9, 0, D)) if rank == 0 else None
    bufs = [torch.zeros(B, 224, 224, 3, dtype=torch.uint8) for _ in range(2)]
    chunks = lambda r: split_range(r * world * B % (D - world * B + 1), r * world * B % (D - world * B + 1)  # noqa
                                   + world * B - 1, world)
    ok, posted = True, {0: plane.scatter_async(src, chunks(0), bufs[0])}
    for r in range(5):
        posted[r + 1] = plane.scatter_async(src, chunks(r + 1), bufs[(r + 1) % 2])
        plane.wait_scatter(posted.pop(r))
        s, e = chunks(r)[rank]
        ok &= np.array_equal(bufs[r % 2].numpy(), synth_images_cpu(9, s, e - s + 1))
    plane.wait_scatter(posted.pop(5))
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_scatter_async_double_buffered_over_gloo():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_scatter_async_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res == {r: True for r in range(world)}


def _bench_pattern_worker(rank, world, port, q):
    """bench.py's round: the forward reads its window start from the broadcast
    descriptor row in place and writes packed (class, prob bits) straight into
    the gather send buffer; rank 0 copies ``gathered_all`` once."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from idunno.parallel.dataplane import QueryPlane, init_from_env, unpack

    env = init_from_env(backend="gloo")
    B, shard_base = 8, rank * 1000
    plane = QueryPlane(env, coordinator=0, max_chunk=B)
    start_dev, send = plane.row_start(), plane.send_buffer[:B]

    def fake_forward():                       # stands in for the captured hipGraph
        s0 = int(start_dev.item()) - shard_base
        idx = torch.arange(s0, s0 + B, dtype=torch.int32) + shard_base
        send[:, 0] = (idx * 7919 + 13) % 1000
        send[:, 1] = torch.full((B,), 0.25).view(torch.int32)

    out = {}
    for q_ in range(4):
        table = [(1, q_ * world + r, r * 1000 + 3 * q_, r * 1000 + 3 * q_ + B - 1) for r in range(world)] \
            if env.rank == 0 else None
        plane.dispatch_device(table, slot=q_)
        fake_forward()
        plane.gather(None, None)
        if env.rank == 0:
            host = plane.gathered_all.clone()
            for r in range(world):
                c, p = unpack(host[r], B)
                for i, (cc, pp) in enumerate(zip(c.tolist(), p.tolist())):
                    out[(q_, table[r][2] + i)] = (cc, pp)
    if env.rank == 0:
        q.put(out)
    if env.distributed:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 8])      # 8: the driver's full-node bench topology
def test_bench_round_pattern_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_bench_pattern_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert len(out) == 4 * world * 8
    for (_q, i), (c, p) in out.items():
        assert c == (i * 7919 + 13) % 1000 and p == 0.25


def _pipelined_worker(rank, world, port, q):
    """bench.py's double-buffered round at N > 1: round q+1's descriptors are
    broadcast into the other slot before round q's forward runs, and round q's
    gather is finished only after round q+1's forward; every slot's results
    must still belong to that slot's round."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from idunno.parallel.dataplane import QueryPlane, init_from_env, unpack

    env = init_from_env(backend="gloo")
    B, rounds = 8, 7
    plane = QueryPlane(env, coordinator=0, max_chunk=B, nbuf=2)

    def table(q_):
        return [(1, q_, 100 * q_ + r * B, 100 * q_ + r * B + B - 1) for r in range(world)]

    def forward(slot):
        s0 = int(plane.row_start_slot(slot).item())
        idx = torch.arange(s0, s0 + B, dtype=torch.int32)
        plane.send_slot(slot)[:B, 0] = (idx * 31 + 5) % 1000
        plane.send_slot(slot)[:B, 1] = torch.full((B,), 0.5).view(torch.int32)

    out, posted, gathers = {}, {}, []

    def finish():
        q_, work = gathers.pop(0)
        plane.wait_work(work)
        if env.rank == 0:
            host = plane.gathered_slot(q_ % 2).clone()
            for r in range(world):
                c, _ = unpack(host[r], B)
                out[(q_, r)] = c.tolist()

    for q_ in range(rounds):
        if q_ not in posted:
            posted[q_] = plane.post_dispatch(table(q_) if env.rank == 0 else None, q_ % 2, q_)
        if q_ + 1 < rounds:
            posted[q_ + 1] = plane.post_dispatch(table(q_ + 1) if env.rank == 0 else None, (q_ + 1) % 2, q_ + 1)
        plane.wait_work(posted.pop(q_))
        forward(q_ % 2)
        if gathers:
            finish()
        gathers.append((q_, plane.post_gather(q_ % 2)))
    while gathers:
        finish()
    if env.rank == 0:
        ok = len(out) == rounds * world and all(
            c == [((table(q_)[r][2] + i) * 31 + 5) % 1000 for i in range(B)] for (q_, r), c in out.items())
        q.put(ok)
    if env.distributed:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 3])
def test_double_buffered_rounds_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert ok is True


def _bucketed_scatter_worker(rank, world, port, q):
    """Bucketed scatter (1 MiB buckets = 6 images, round-robin over the peers):
    every rank's shard arrives byte-exact, uneven shard sizes included, for the
    async double-buffered path and the synchronous path."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist

    from idunno.parallel.dataplane import NO_WORK, QueryPlane, init_from_env
    from idunno.runtime.data import synth_images_cpu
    from idunno.runtime.scheduler import split_range

    env = init_from_env(backend="gloo")
    plane = QueryPlane(env, coordinator=0, max_chunk=20)
    plane.scatter_bucket_bytes = 1 << 20
    assert plane._bucket_rows(224 * 224 * 3) == 6
    B = 20
    src = torch.from_numpy(synth_images_cpu(11, 0, world * B + 13)) if rank == 0 else None
    ok = True
    bufs = [torch.zeros(B, 224, 224, 3, dtype=torch.uint8) for _ in range(2)]
    rounds = [split_range(0, world * B - 1, world), split_range(13, 13 + world * B - 8, world)]
    posted = [plane.scatter_async(src, ch, bufs[i]) for i, ch in enumerate(rounds)]
    for i, ch in enumerate(rounds):
        plane.wait_scatter(posted[i])
        s, e = ch[rank]
        ok &= np.array_equal(bufs[i][:e - s + 1].numpy(), synth_images_cpu(11, s, e - s + 1))
    # synchronous scatter, one idle rank
    table = None
    if rank == 0:
        chunks = split_range(100, 100 + 7 * (world - 1) + 4, world - 1) if world > 1 else [(100, 104)]
        table = [(1, 0, s, e) for s, e in chunks] + [(1, 0, 0, NO_WORK)] * (world - len(chunks))
        imgs = torch.from_numpy(synth_images_cpu(11, 100, chunks[-1][1] - 99))
    row = plane.dispatch(table)
    got = plane.scatter(imgs if rank == 0 else None, table, row)
    if row[3] == NO_WORK:
        ok &= got is None
    else:
        ok &= np.array_equal(got.numpy(), synth_images_cpu(11, row[2], row[3] - row[2] + 1))
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_bucketed_scatter_byte_exact_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_bucketed_scatter_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res == {r: True for r in range(world)}


def test_scatter_bucket_split_round_robin():
    """The root's op list: bucket k of every peer before bucket k+1 of any, and
    each peer's pieces tile its rows exactly (CPU, no process group)."""
    import types

    from idunno.parallel.dataplane import QueryPlane

    plane = QueryPlane.__new__(QueryPlane)
    plane.coord, plane.group, plane.scatter_bucket_bytes = 0, None, 3 * 10
    imgs = torch.arange(40 * 10, dtype=torch.uint8).view(40, 10)
    seen = []
    import idunno.parallel.dataplane as dp
    real = dp.dist.P2POp
    dp.dist.P2POp = lambda op, t, peer, group: types.SimpleNamespace(t=t, peer=peer)
    try:
        ops = plane._send_ops(imgs, {1: (0, 6), 2: (7, 8), 3: (9, 17)})
        rops = plane._recv_ops(torch.zeros(7, 10, dtype=torch.uint8))
    finally:
        dp.dist.P2POp = real
    seen = [(o.peer, o.t.shape[0]) for o in ops]
    assert seen == [(1, 3), (2, 2), (3, 3), (1, 3), (3, 3), (1, 1), (3, 3)]
    assert [o.t.shape[0] for o in rops] == [3, 3, 1]


def test_connect_aborts_on_failed_check():
    """ElasticGroup._connect (the RCCL communicator set-up of form()): a set-up
    blocked on a dead member ends when check() fails -- the communicator is
    aborted from a helper thread, which releases the blocked connect -- and a
    set-up that finishes returns True."""
    import threading
    import time

    import torch

    from idunno.parallel.elastic import ElasticGroup

    class FakePg:
        def __init__(self):
            self.released = threading.Event()
            self.aborted = False

        def connect(self, device):          # blocks like a bootstrap waiting on a dead rank
            self.released.wait(30)

        def abort(self):
            self.aborted = True
            self.released.set()

    g = ElasticGroup(torch.device("cpu"), timeout_s=20)
    pg = FakePg()
    t0 = time.monotonic()
    alive = {"ok": True}
    threading.Timer(0.2, lambda: alive.update(ok=False)).start()
    assert g._connect(pg, pg.connect, lambda: alive["ok"]) is False
    assert time.monotonic() - t0 < 5
    assert g.join_aborters(5) and pg.aborted
    ok_pg = FakePg()
    ok_pg.released.set()
    assert g._connect(ok_pg, ok_pg.connect, lambda: True) is True and not ok_pg.aborted
