"""Unit tests of the control-plane building blocks (CPU, no GPU)."""
import json
import os
import socket
import threading
import time
import types

import numpy as np
import pytest

from idunno.config import ClusterConfig
from idunno.runtime import messages as M
from idunno.runtime.jobstate import JobState
from idunno.runtime.sdfs import VERSION_DELIM, SdfsStore, ring_placement, stable_hash
from idunno.runtime.transport import InMemoryNetwork, TcpTransport, TransportError, wait_for


# -- framing ---------------------------------------------------------------------
def test_frame_roundtrip_and_partial_reads():
    msgs = [{"t": M.Type.RESULT, "cls": np.arange(5000, dtype=np.int32).tobytes(), "q": i} for i in range(3)]
    stream = b"".join(M.encode(m) for m in msgs)
    rd = M.FrameReader()
    out = []
    for i in range(0, len(stream), 777):           # arbitrary fragmentation
        out += rd.feed(stream[i:i + 777])
    assert [o["q"] for o in out] == [0, 1, 2]
    assert np.frombuffer(out[2]["cls"], np.int32)[-1] == 4999  # > 4096 bytes: no truncation (A4)


# -- transports -------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_tcp_request_reply_and_unreachable():
    base = _free_port()
    cfg = ClusterConfig(base_port=base, num_nodes=2)
    a = TcpTransport("node00", cfg.address, cfg.address("node00"))
    b = TcpTransport("node01", cfg.address, cfg.address("node01"))
    a.start(lambda m: {"echo": m["x"] * 2})
    b.start(lambda m: None)
    try:
        r = b.request("node00", {"t": "X", "x": 21}, timeout=2)
        assert r["echo"] == 42 and r["src"] == "node00"
        a.close()
        with pytest.raises(TransportError):
            b.request("node00", {"t": "X", "x": 1}, timeout=0.5)
        # the peer is gone: within a couple of sends the refused reconnect is reported
        assert wait_for(lambda: not b.send("node00", {"t": "X", "x": 1}), 2)
    finally:
        a.close()
        b.close()


def test_inmemory_faults():
    net = InMemoryNetwork()
    got = []
    a, b = net.transport("a"), net.transport("b")
    a.start(lambda m: None)
    b.start(lambda m: got.append(m["i"]))
    assert a.send("b", {"t": "X", "i": 1})
    net.partition("a", "b")
    assert a.send("b", {"t": "X", "i": 2})          # silently lost
    net.heal()
    net.crash("b")
    assert not a.send("b", {"t": "X", "i": 3})      # refused
    assert wait_for(lambda: got == [1], 1)


# -- SDFS store / placement ----------------------------------------------------------
def test_stable_placement():
    ring = [f"node{i:02d}" for i in range(8)]
    p1 = ring_placement("images/shard_00001", ring, 4)
    assert p1 == ring_placement("images/shard_00001", ring, 4)   # stable across processes (A8)
    assert len(set(p1)) == 4
    assert stable_hash("a") == 3904355907                          # crc32


def test_store_versions(tmp_path):
    st = SdfsStore(str(tmp_path))
    st.write("dir/f.txt", 1, b"a")
    st.write("dir/f.txt", 2, b"bb")
    assert st.versions("dir/f.txt") == [1, 2]
    assert st.read("dir/f.txt") == b"bb" and st.read("dir/f.txt", 1) == b"a"
    assert st.files() == ["dir/f.txt"]
    assert st.unlink("dir/f.txt") == 2 and st.files() == []
    with pytest.raises(ValueError):
        st.write("../etc/passwd", 1, b"x")


# -- job state --------------------------------------------------------------------------
def test_jobstate_tables_and_views(tmp_path):
    clock = [100.0]
    js = JobState(clock=lambda: clock[0])
    q = js.new_query_number("resnet18")
    js.assign("resnet18", q, [("node01", 0, 79), ("node02", 80, 159)])
    assert js.cvm().startswith("{'node01': [('resnet18', 1, 0, 79)]")
    clock[0] = 101.0
    assert js.record_result("resnet18", q, "node01", 0, 79, np.arange(80) % 1000, np.full(80, 0.25))
    assert not js.record_result("resnet18", q, "node01", 0, 79, np.zeros(80), np.zeros(80))  # idempotent
    assert js.images_done("resnet18") == 80                                              # A3: end-start+1
    assert ("node01", 0, 79, "f", 100.0, 101.0) in js.worker_set[("resnet18", 1)]
    assert "node01" not in js.working_vm_set
    clock[0] = 102.0
    js.record_result("resnet18", q, "node02", 80, 159, np.ones(80), np.full(80, 0.5))
    assert js.finished_queries["resnet18"] == 1
    assert js.query_latency["resnet18"] == [2.0]
    c1 = js.c1()
    assert "Resnet18 finished inference is 160" in c1
    c2 = js.c2()
    assert c2.startswith("model resnet18 processing time") and "average" in c2
    path = tmp_path / "result.txt"
    js.c4(str(path))
    d = json.loads(path.read_text())
    first = d["resnet18 1"][0]
    assert first.startswith("[('test_0.JPEG', 'class_0', 0.25)")
    # snapshot / restore round trip through msgpack
    import msgpack

    snap = msgpack.unpackb(msgpack.packb(js.snapshot()), raw=False, strict_map_key=False)
    js2 = JobState()
    js2.restore(snap)
    assert js2.images_done("resnet18") == 160
    assert js2.inference_result_list() == js.inference_result_list()


def test_jobstate_reassign_and_pending():
    js = JobState()
    js.assign("alexnet", 1, [("node03", 0, 99)])
    js.reassign("node03", "node04", ("alexnet", 1, 0, 99))
    assert js.chunks_of("node04") == [("alexnet", 1, 0, 99)] and js.chunks_of("node03") == []
    assert [p[2] for p in js.pending()] == ["node04"]


def test_jobstate_dedupes_images_across_chunk_splits():
    """A query re-dispatched with a different chunk split (promoted standby
    resuming a job under its reserved query number) counts each image once."""
    js = JobState()
    jid = js.add_job("resnet18", 0, 999, 400)            # 3 queries -> numbers 1, 2, 3 reserved
    assert [js.job_query_number(jid, s) for s in (0, 400, 800)] == [1, 2, 3]
    assert js.new_query_number("resnet18") == 4
    cls = np.zeros(400, np.int32)
    prob = np.ones(400, np.float32)
    js.assign("resnet18", 1, [("a", 0, 199), ("b", 200, 399)])
    assert js.record_result("resnet18", 1, "a", 0, 199, cls[:200], prob[:200])
    # the same query re-issued over three workers: only images 200..399 are new
    js.assign("resnet18", 1, [("c", 0, 132), ("d", 133, 265), ("e", 266, 399)])
    assert not js.record_result("resnet18", 1, "c", 0, 132, cls[:133], prob[:133])
    assert js.record_result("resnet18", 1, "d", 133, 265, cls[:133], prob[:133])
    assert js.record_result("resnet18", 1, "e", 266, 399, cls[:134], prob[:134])
    assert js.record_result("resnet18", 1, "b", 200, 399, cls[:200], prob[:200]) is False
    assert js.images_done("resnet18") == 400
    assert js.finished_queries["resnet18"] == 1
    # the same images under a NEW query number are new work (repeated queries count)
    js.assign("resnet18", 5, [("a", 0, 399)])
    assert js.record_result("resnet18", 5, "a", 0, 399, cls, prob)
    assert js.images_done("resnet18") == 800


def test_standby_reopens_chunks_it_holds_no_results_for():
    coord, standby = JobState(), JobState()
    cls, prob = np.zeros(80, np.int32), np.ones(80, np.float32)
    coord.assign("alexnet", 1, [("a", 0, 79), ("b", 80, 159)])
    standby.record_result("alexnet", 1, "a", 0, 79, cls, prob)        # dual-sent, arrived
    coord.record_result("alexnet", 1, "a", 0, 79, cls, prob)
    coord.record_result("alexnet", 1, "b", 80, 159, cls, prob)        # reached the coordinator only
    standby.restore(coord.snapshot(include_results=False), keep_results=True)
    assert standby.pending() == []                                    # the snapshot says all done
    assert standby.reopen_unheld() == 1
    assert [(w, s, e) for _m, _q, w, s, e, _t in standby.pending()] == [("b", 80, 159)]
    assert standby.record_result("alexnet", 1, "c", 80, 159, cls, prob)
    assert standby.images_done("alexnet") == 160 and standby.pending() == []
    # re-dispatch with the SAME chunk boundaries as an answered original: the
    # late duplicate answer closes the new entry (and is not counted)
    standby.assign("alexnet", 1, [("d", 0, 79)])
    assert standby.record_result("alexnet", 1, "d", 0, 79, cls, prob) is False
    assert standby.pending() == [] and standby.images_done("alexnet") == 160


def test_config_env_and_file(tmp_path):
    p = tmp_path / "c.json"
    p.write_text(json.dumps({"num_nodes": 4, "heartbeat_period_s": 0.1}))
    cfg = ClusterConfig.load(str(p), env={"IDUNNO_FAILURE_TIMEOUT_S": "0.7", "IDUNNO_REPLICATION": "3"},
                             base_port=20000)
    assert cfg.num_nodes == 4 and cfg.heartbeat_period_s == 0.1 and cfg.failure_timeout_s == 0.7
    assert cfg.replication == 3 and cfg.base_port == 20000
    assert cfg.standby_name == "node03" and cfg.address("node02") == ("127.0.0.1", 20002)
    with pytest.raises(KeyError):
        cfg.update(bogus=1)


def test_round_finalize_reruns_range_guard_rows_only():
    """RoundPlane._finalize: a row whose split forward left fp16's range (class
    -2 inside its chunk) goes back to its member as a TCP JOB (f32 rerun); rows
    with stale negatives only past their chunk's end are ingested as usual; the
    scheduler gets the round's (chunk size, seconds) points of each model in one
    call (observe_chunks), every member's header included."""
    import numpy as np

    from idunno.config import ClusterConfig
    from idunno.parallel.elastic import HDR_ROWS, MODEL_IDS
    from idunno.runtime.rounds import RoundPlane, _Round

    mc, W = 16, 3
    arr = np.zeros((W, mc + HDR_ROWS, 2), np.int32)
    arr[:, :mc, 0] = np.arange(mc)[None, :] + 100 * np.arange(W)[:, None]
    arr[:, :mc, 1] = np.float32(0.5).view(np.int32)
    arr[1, 3, 0] = -2                          # inside member 1's chunk (4 images): rerun
    arr[2, 10, 0] = -2                         # member 2's chunk has 6 images: stale tail, ignored
    mid = MODEL_IDS["resnet18"]
    for i, (us, cnt) in enumerate([(400, 4), (800, 4), (600, 6)]):
        arr[i, mc] = (us, mid)
        arr[i, mc + 1] = (cnt, 1)

    class G:
        max_chunk = mc
        standby_rank = -1

        def collect(self, seq, work, check):
            return arr

    sent, ingested, observed = [], [], []
    node = types.SimpleNamespace(
        name="node00", standby="node00",
        sched=types.SimpleNamespace(observe_chunks=lambda m, pts, b: observed.append((m, list(pts), b))),
        _send_job=lambda *a: sent.append(a), _ingest_round=lambda recs, now, seq: ingested.extend(recs),
        membership=types.SimpleNamespace(is_alive=lambda n: True))
    rp = RoundPlane.__new__(RoundPlane)
    rp.node, rp.group, rp.cfg = node, G(), ClusterConfig()
    rp.host_s = rp.host_wait_s = rp.host_cpu_s = 0.0
    rp.rounds_done = 0
    table = [(mid, 7, 0, 3), (mid, 7, 4, 7), (mid, 7, 8, 13)]
    rp._finalize(_Round(1, [], table), ("node00", "node01", "node02"), None)
    assert sent == [("node01", "resnet18", 7, 4, 7)]
    assert [(r[2], r[3], r[4]) for r in ingested] == [("node00", 0, 3), ("node02", 8, 13)]
    assert list(ingested[1][5]) == list(range(200, 206)) and np.all(ingested[1][6] == 0.5)
    assert len(observed) == 1 and observed[0][0] == "resnet18"
    pts = observed[0][1]
    assert [n for n, _ in pts] == [4, 4, 6]
    assert all(abs(t - u * 1e-6) < 1e-12 for (_, t), u in zip(pts, (400, 800, 600)))
    assert observed[0][2] == rp.cfg.batch_for("resnet18")


def test_send_frame_falls_back_when_the_socket_buffer_is_full():
    """transport._send_frame: the GIL-holding non-blocking send takes what fits
    and the rest goes through sendall; a closed peer raises OSError."""
    from idunno.runtime.transport import _send_frame

    a, b = socket.socketpair()
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4096)
    data = os.urandom(4 << 20)                     # far larger than the send buffer
    got = bytearray()

    def rd():
        while len(got) < len(data):
            chunk = b.recv(1 << 16)
            if not chunk:
                break
            got.extend(chunk)
    th = threading.Thread(target=rd)
    th.start()
    _send_frame(a, b"x" * 10)                       # fits: one non-blocking send
    _send_frame(a, data[10:])
    th.join(30)
    assert bytes(got) == b"x" * 10 + data[10:]
    b.close()
    with pytest.raises(OSError):
        for _ in range(64):                         # the peer is gone: EPIPE / ECONNRESET
            _send_frame(a, data[:1 << 16])
    a.close()


def test_round_batch_announce_and_member_unpack():
    """Coordinator: with a backlog of full rounds, up to ANNOUNCE_ROUNDS
    descriptor tables share ONE multicast frame; a partial round after the
    first stays queued (another job's query may still join it).  Member: a
    batch frame is unpacked into per-seq descriptors."""
    import threading as th
    from collections import deque

    from idunno.config import ClusterConfig
    from idunno.runtime.rounds import RoundPlane, _Query

    members = ("node00", "node01", "node02", "node03")
    frames = []
    node = types.SimpleNamespace(
        name="node00", transport=types.SimpleNamespace(multicast=lambda d, m: frames.append((list(d), m)) or []),
        state=types.SimpleNamespace(active_models=lambda: {"resnet18"}),
        membership=types.SimpleNamespace(alive=lambda: list(members)))
    rp = RoundPlane.__new__(RoundPlane)
    rp.node, rp.cfg, rp.cv = node, ClusterConfig(), th.Condition()
    rp.group = types.SimpleNamespace(epoch=5)
    rp._queue, rp._built_for, rp._next_seq = deque(), None, 0
    rp.host_send_s, rp.announce_frames = 0.0, 0
    full = lambda q: _Query("resnet18", q, {m: (100 * q + i, 100 * q + i) for i, m in enumerate(members)}, members)  # noqa: E731
    half = _Query("alexnet", 9, {"node00": (0, 0), "node01": (1, 1)}, members)
    rp._queue.extend([full(1), full(2), half, full(3)])
    rounds = rp._build_rounds(members)
    assert [r.seq for r in rounds] == [0, 1]                  # the partial 3rd round is not committed
    assert [q.qnum for q in rp._queue] == [9, 3]              # ... and keeps its queue position
    rp._announce(rounds, members)
    assert len(frames) == 1 and frames[0][0] == list(members[1:])
    msg = frames[0][1]
    from idunno.parallel.elastic import MODEL_IDS
    rid = MODEL_IDS["resnet18"]
    assert [s for s, _ in msg["batch"]] == [0, 1] and msg["batch"][1][1][2] == [rid, 2, 202, 202]
    # a partial FIRST round is built as before (posted at once); a full one may follow it
    rounds = rp._build_rounds(members)
    assert [r.seq for r in rounds] == [2, 3] and [q.qnum for q in rounds[0].queries] == [9]
    assert not rp._queue
    # member side
    mem = RoundPlane.__new__(RoundPlane)
    mem.cv, mem.epoch, mem._round_msgs, mem.members = th.Condition(), 5, {}, list(members)
    staged = []
    mem.node = types.SimpleNamespace(name="node02", source=types.SimpleNamespace(prefetch=lambda s, e: staged.append((s, e))))
    mem.on_round(dict(msg, src="node00"))
    assert staged == [(102, 102), (202, 202)]          # its announced chunks start staging at once
    assert sorted(mem._round_msgs) == [(5, 0), (5, 1)]
    assert mem._round_msgs[(5, 1)]["rows"][3] == [rid, 2, 203, 203]


def test_executor_trims_cache_only_when_no_collective_can_pend(monkeypatch):
    """HipExecutor._capture frees the allocator cache after a new capture only
    while ``trim_ok`` says no collective can be pending: hipFree waits for every
    kernel on the device with the interpreter lock held, and behind a gather
    stuck on a dead peer it stalled the whole node (8-rank RCCL rehearsal)."""
    import torch

    from idunno.runtime.executor import HipExecutor
    from idunno.runtime.rounds import RoundPlane

    calls = []
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: calls.append(1))
    ex = HipExecutor.__new__(HipExecutor)
    ex.graphs_broken = False
    r = types.SimpleNamespace(_graphs={})

    def cap():
        r._graphs[len(r._graphs)] = object()
        return "replay"

    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda d=None: 10 << 30)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda d=None: 1 << 30)
    ex.device = "cuda:0"
    ex._trim_wanted = False
    ex.trim_slack_bytes = 16 << 30
    seen = []
    ex.trim_ok = lambda need: seen.append(need) or False
    assert ex._capture(r, cap) == "replay" and calls == [] and seen == [False]
    ex.trim_slack_bytes = 2 << 30                        # 9 GiB unused > 2 GiB slack: a need
    assert ex._capture(r, cap) == "replay" and calls == [] and seen == [False, True]
    assert ex._trim_wanted                               # owed: retried at a quiet point
    ex.trim_ok = lambda need: True
    ex.maybe_trim()
    assert calls == [1] and not ex._trim_wanted
    ex.maybe_trim()
    assert calls == [1]                                  # nothing owed
    assert ex._capture(r, lambda: "hit") == "hit" and calls == [1]      # no new graph: no trim

    import threading
    from collections import deque

    class Work:
        def __init__(self, done):
            self.done = done

        def is_completed(self):
            return self.done

    rp = RoundPlane.__new__(RoundPlane)
    rp._thread = threading.current_thread()              # as if on the round driver
    rp._inflight = deque()
    def group(formed, members, aborting=False):
        return types.SimpleNamespace(formed=formed, members=members, aborting=lambda: aborting)

    rp.group = group(False, [])
    assert rp.collectives_quiet()
    rp.group = group(True, ["a"])
    assert rp.collectives_quiet()                        # a one-member (solo) epoch
    rp.group = group(True, ["a", "b"])
    assert not rp.collectives_quiet() and rp.collectives_quiet(need=True)
    rp._inflight.append([3, Work(False), None, False])    # a gather still in flight: it may never end
    assert not rp.collectives_quiet(need=True)
    rp._inflight[0][1].done = True
    assert rp.collectives_quiet(need=True)
    rp._thread = None                                    # not the driver thread: it may post meanwhile
    assert not rp.collectives_quiet(need=True)
    rp.group = group(False, [], aborting=True)
    assert not rp.collectives_quiet(need=True)           # an aborted communicator still tearing down
