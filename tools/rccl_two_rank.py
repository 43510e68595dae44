#!/usr/bin/env python3
"""Two RCCL ranks on ONE GPU (the runtime's RCCL paths with world > 1 on a
one-GPU box).  RCCL refuses two ranks of one host on one device ("Duplicate
GPU detected", keyed by host hash + bus id); giving each rank its own
NCCL_HOSTID makes them distinct "hosts", so the communicator forms over RCCL's
socket transport on loopback instead of xGMI P2P.  The collectives, the
ProcessGroupNCCL / ElasticGroup code and abort() are RCCL's own; only the
transport differs from the 8-GPU node.

Checks (rank 0 prints one JSON line of results):
  1. QueryPlane on the default group: descriptor broadcast, top-1 gather, and
     the bucketed scatter (batch_isend_irecv) byte-exact;
  2. ElasticGroup epoch (ProcessGroupNCCL on a PrefixStore, eager connect):
     double-buffered gather rounds to the coordinator AND the standby root;
  3. the peer dies (os._exit) with a gather posted: rank 0's wait sees the
     liveness check fail, abort_async() ends the communicator, a new solo epoch
     forms.

usage: python tools/rccl_two_rank.py            (spawns both ranks, exit code = rank 0's)
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_main(rank: int, port: int, eport: int, marker: str) -> int:
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), NCCL_HOSTID=f"idunno-rank{rank}", NCCL_SOCKET_IFNAME="lo")
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from idunno.parallel.dataplane import NO_WORK, QueryPlane, init_from_env, unpack
    from idunno.parallel.elastic import HDR_ROWS, ElasticGroup, RoundAbandoned

    res = {}
    env = init_from_env(backend="nccl", timeout_s=120)
    assert env.backend == "nccl" and env.world == 2
    dev = env.device
    res["backend"] = dist.get_backend()
    # 1. QueryPlane: broadcast + gather + bucketed scatter
    plane = QueryPlane(env, coordinator=0, max_chunk=512)
    table = [(1, 7, 0, 299), (1, 7, 300, 499)] if rank == 0 else None
    row = plane.dispatch(table)
    n = row[3] - row[2] + 1
    cls = torch.arange(row[2], row[3] + 1, device=dev, dtype=torch.int32)
    prob = torch.full((n,), 0.5 + rank, device=dev)
    g = plane.gather(cls, prob)
    if rank == 0:
        c1, p1 = unpack(g[1], 200)
        res["gather_ok"] = bool(torch.equal(c1.cpu(), torch.arange(300, 500, dtype=torch.int32))
                                and bool((p1 == 1.5).all()))
    plane.scatter_bucket_bytes = 1 << 20                # several buckets per peer shard
    shape = (16, 64, 64, 3)                             # 196 KB per image
    imgs = None
    if rank == 0:
        imgs = (torch.arange(40 * 64 * 64 * 3, device=dev) % 251).to(torch.uint8).view(40, *shape[1:])
    out = torch.empty((24, *shape[1:]), dtype=torch.uint8, device=dev)
    reqs = plane.scatter_async(imgs, [(0, 15), (16, 39)], out)
    plane.wait_scatter(reqs)
    torch.cuda.synchronize()
    want = (torch.arange(40 * 64 * 64 * 3, device=dev) % 251).to(torch.uint8).view(40, *shape[1:])
    ok = torch.equal(out[:16], want[:16]) if rank == 0 else torch.equal(out[:24], want[16:40])
    okt = torch.tensor([int(ok)], device=dev)
    dist.all_reduce(okt)
    res["scatter_ok"] = int(okt.item()) == 2
    dist.barrier()
    dist.destroy_process_group()

    # 2. ElasticGroup epoch over RCCL, gather pairs to coordinator + standby
    grp = ElasticGroup(dev, backend="nccl", timeout_s=60, op_timeout_s=40, max_chunk=256)
    me = f"node{rank}"
    assert grp.form(me, ["node0", "node1"], 1, "127.0.0.1", eport, standby="node1")
    res["epoch_backend"] = grp.describe().get("backend")
    rounds_ok = True
    for seq in range(6):
        send = grp.send_buffer(seq)
        send[:10, 0] = torch.arange(10, device=dev, dtype=torch.int32) + 100 * rank + seq
        grp.header(seq)[0, 0] = seq
        work = grp.post_gather(seq)
        h = grp.collect(seq, work)                 # both ranks are roots (coordinator, standby)
        for r in range(2):
            rounds_ok &= bool((h[r, :10, 0] == [100 * r + seq + i for i in range(10)]).all())
            rounds_ok &= int(h[r, grp.max_chunk, 0]) == seq
        grp.release(work)
    res["rounds_ok"] = rounds_ok
    # 3. the peer dies with a gather posted; rank 0 notices through its check, aborts
    if rank == 1:
        open(marker, "w").close()
        time.sleep(0.5)
        os._exit(0)
    while not os.path.exists(marker):
        time.sleep(0.05)
    time.sleep(1.5)                                 # the peer is gone
    work = grp.post_gather(6)
    t0 = time.perf_counter()
    dead = {"t": time.perf_counter() + 0.3}

    def check():
        if time.perf_counter() > dead["t"]:
            raise RoundAbandoned("peer node1 failed")

    try:
        grp.wait(work, check)
        res["abandoned"] = False
    except RoundAbandoned:
        res["abandoned"] = True
    if os.environ.get("RCCL2_STREAM_DEP") == "1":
        work.wait()                                 # the compute stream now depends on the dead gather
    grp.abort_async()
    res["abort_returned"] = grp.join_aborters(60)
    res["abort_s"] = round(time.perf_counter() - t0, 3)
    # GPU work queued on the compute stream after the abort must run: the aborted
    # collective may not hold the stream (a stream dependency on it would stall
    # every later forward until the backend's timeout)
    t1 = time.perf_counter()
    x = torch.ones(1 << 20, device=dev)
    res["after_abort_sum"] = float((x * 2).sum().item())
    res["after_abort_s"] = round(time.perf_counter() - t1, 3)
    assert grp.form(me, ["node0"], 2, "127.0.0.1", _port())      # survivors re-form (solo)
    res["reformed_world"] = grp.world
    print(json.dumps(res), flush=True)
    ok = all(res.get(k) for k in ("gather_ok", "scatter_ok", "rounds_ok", "abandoned", "abort_returned"))
    return 0 if ok else 1


def main() -> int:
    if len(sys.argv) > 1 and sys.argv[1] == "--rank":
        return rank_main(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
    port, eport = _port(), _port()
    marker = f"/tmp/idunno_rccl2_{os.getpid()}"
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank", str(r), str(port), str(eport),
                               marker]) for r in range(2)]
    try:
        rc0 = procs[0].wait(timeout=240)
        procs[1].wait(timeout=30)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        if os.path.exists(marker):
            os.unlink(marker)
    return rc0


if __name__ == "__main__":
    sys.exit(main())
