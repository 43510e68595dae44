"""Fake multi-node cluster tests: N nodes in one process on the in-memory
transport (or TCP), deterministic FakeExecutor.  Covers membership, failure
detection, chunk re-dispatch, SDFS replication/re-replication, hot-standby
failover, concurrent jobs and the shell (SURVEY.md §4 "fake multi-node")."""
import json
import time

import numpy as np
import pytest

from idunno.runtime.cluster import LocalCluster
from idunno.runtime.shell import Shell
from idunno.runtime.transport import wait_for

FAST = dict(heartbeat_period_s=0.05, failure_timeout_s=1.0, metadata_period_s=0.1, rpc_timeout_s=2.0)


def expected_cls(model, s, e):
    idx = np.arange(s, e + 1)
    salt = 7 if model == "alexnet" else 13
    return (idx * 7919 + salt) % 1000


def check_results(client, model, s, e):
    res = client.view("c4")["results"]
    got = {}
    for k, chunks in res.items():
        if not k.startswith(model + " "):
            continue
        for ch in chunks:
            for name, cat, p in eval(ch):  # reference string format
                got[int(name[5:-5])] = int(cat.split("_")[1])
    exp = expected_cls(model, s, e)
    missing = [i for i in range(s, e + 1) if i not in got]
    assert not missing, f"missing {len(missing)} images, e.g. {missing[:5]}"
    assert all(got[i] == exp[i - s] for i in range(s, e + 1))


@pytest.fixture
def cluster():
    c = LocalCluster(num_nodes=6, **FAST).start()
    yield c
    c.stop()


def test_membership_converges(cluster):
    coord = cluster.coordinator()
    assert coord.name == "node00"
    assert len(coord.membership.alive()) == 6
    n3 = cluster.nodes["node03"]
    assert wait_for(lambda: len(n3.membership.alive()) == 6, 2)   # JOIN forwarded + PING merge


def test_query_end_to_end(cluster):
    cl = cluster.client()
    r = cl.inference(0, 999, "resnet18")
    assert [x["qnum"] for x in r] == [1, 2, 3]
    assert [len(x["plan"]) for x in r] == [6, 6, 6]
    s = cl.wait_idle(10, {"resnet18": 1000})
    assert s["done"]["resnet18"] == 1000 and s["pending"] == 0
    check_results(cl, "resnet18", 0, 999)
    assert "Resnet18 finished inference is 1000" in cl.view("c1")["text"]
    assert "model resnet18 processing time" in cl.view("c2")["text"]


def test_worker_failure_redispatch(cluster):
    cl = cluster.client("node05")
    for n in ("node02", "node03"):
        cluster.nodes[n].extra_delay_s = 0.6
    cl.inference(0, 399, "alexnet")
    time.sleep(0.1)
    cluster.crash("node02")
    s = cl.wait_idle(10, {"alexnet": 400})
    assert s["done"]["alexnet"] == 400
    coord = cluster.coordinator()
    assert "node02" not in coord.membership.alive()
    check_results(cl, "alexnet", 0, 399)
    assert "node02" not in coord.state.cvm()


def test_sdfs_ops_and_rereplication(cluster, tmp_path):
    n = cluster.nodes["node04"]
    f = tmp_path / "local.txt"
    f.write_text("v1")
    sh = Shell(n, cluster.client("node04"))
    assert "version 1" in sh.execute(f"put {f} data/a.txt")
    f.write_text("v2")
    assert "version 2" in sh.execute(f"put {f} data/a.txt")
    reps = n.sdfs.ls("data/a.txt")
    assert len(reps) == 4
    out = tmp_path / "got.txt"
    assert sh.execute(f"get data/a.txt {out}") == "ok" and out.read_text() == "v2"
    gv = tmp_path / "gv.txt"
    assert "wrote 2" in sh.execute(f"get-versions data/a.txt 5 {gv}")
    txt = gv.read_text()
    assert txt == f"{VERSION}version2{VERSION}\nv2{VERSION}version1{VERSION}\nv1"
    holder = [r for r in reps if r not in ("node00", "node04")][0]
    cluster.crash(holder)
    assert wait_for(lambda: holder not in n.sdfs.ls("data/a.txt") and len(n.sdfs.ls("data/a.txt")) == 4, 5)
    new = [r for r in n.sdfs.ls("data/a.txt") if r not in reps][0]
    assert cluster.nodes[new].sdfs.store.versions("data/a.txt") == [1, 2]
    assert sh.execute("delete data/a.txt") == "deleted"
    assert all(not cluster.nodes[r].sdfs.store.versions("data/a.txt") for r in n.sdfs.ls("data/a.txt") or reps
               if cluster.nodes[r].alive_flag)
    assert "not found" in sh.execute(f"get data/a.txt {out}")


VERSION = "#" * 30


def test_coordinator_failover_mid_job(cluster):
    cl = cluster.client("node03")
    for n in cluster.nodes.values():
        n.extra_delay_s = 0.3
    cl.inference(0, 799, "resnet18")
    time.sleep(0.25)                       # chunks in flight; let a METADATA push land
    cluster.crash("node00")
    standby = cluster.nodes["node05"]
    assert wait_for(lambda: standby.is_coordinator, 5)
    assert standby.membership.epoch == 1
    assert wait_for(lambda: all(cluster.nodes[n].membership.master == "node05"
                                for n in ("node01", "node02", "node03", "node04")), 3)
    for n in cluster.nodes.values():
        n.extra_delay_s = 0.0
    cl.inference(800, 1199, "resnet18")    # new queries go to the promoted standby
    s = cl.wait_idle(10, {"resnet18": 1200})
    assert s["done"]["resnet18"] == 1200, s
    check_results(cl, "resnet18", 0, 1199)


def test_concurrent_jobs_fair_share(cluster):
    coord = cluster.coordinator()
    coord.sched.observe("alexnet", 6.0)
    coord.sched.observe("resnet18", 9.0)
    coord.cfg.worker_budget = 6
    coord.sched.budget = 6
    for n in cluster.nodes.values():
        n.extra_delay_s = 0.2
    cl = cluster.client()
    ra = cl.submit("alexnet", 0, 499)
    assert len(ra["plan"]) == 6            # a job running alone owns the whole budget
    rr = cl.submit("resnet18", 0, 399)
    ra2 = cl.submit("alexnet", 500, 999)
    # both jobs active: time shares 6 s / 9 s -> the slower model gets more
    # workers (reference formula, mp4_machinelearning.py:509-514): 4 vs 2
    assert len(rr["plan"]) == 4 and len(ra2["plan"]) == 2
    for n in cluster.nodes.values():
        n.extra_delay_s = 0.0
    cl.wait_idle(10, {"alexnet": 1000, "resnet18": 400})


def test_shell_commands(cluster, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    n = cluster.nodes["node02"]
    sh = Shell(n, cluster.client("node02"))
    assert "node00" in sh.execute("list_mem")
    assert sh.execute("list_self").startswith("127.0.0.1:")
    assert "coordinator: node00" in sh.execute("list_master")
    assert sh.execute("inference 0 9") == "Error: missing or too many inference parameter ."
    assert sh.execute("bogus") == "Invalid input. Please try again"
    assert "submitting" in sh.execute("inference 0 99 resnet")
    cluster.client("node02").wait_idle(5, {"resnet18": 100})
    assert "('node" in sh.execute("cq")
    c4 = sh.execute("c4")
    assert "test_0.JPEG" in c4 and json.loads((tmp_path / "result.txt").read_text())
    assert sh.execute("get-versions x 0 y").startswith("Error")
    assert sh.execute("dataset 10 10") == "put 1 shards"
    assert "started" in sh.execute("grep started")
    # fault injection by rank index or name
    assert sh.execute("delay-rank 3 0.25") == "sent"
    assert wait_for(lambda: cluster.nodes["node03"].extra_delay_s == 0.25, 3)
    assert sh.execute("delay node03 0") == "sent"
    assert wait_for(lambda: cluster.nodes["node03"].extra_delay_s == 0.0, 3)
    assert sh.execute("kill-rank 4") == "sent"
    assert wait_for(lambda: "node04" not in cluster.coordinator().membership.alive(), 3)
    assert sh.execute("kill-coordinator x") == "Error: missing or too many kill-coordinator parameter ."
    assert sh.execute("leave") == "left"
    assert wait_for(lambda: "node02" not in cluster.coordinator().membership.alive(), 3)
    assert sh.execute("join") == "joined"
    assert wait_for(lambda: "node02" in cluster.coordinator().membership.alive(), 3)


def test_tcp_cluster_small():
    from test_multiprocess import _base_port

    c = LocalCluster(num_nodes=3, transport="tcp", base_port=_base_port(3), **FAST).start()
    try:
        cl = c.client()
        cl.inference(0, 299, "alexnet")
        st = cl.wait_idle(10, {"alexnet": 300})
        assert st["done"]["alexnet"] == 300
        check_results(cl, "alexnet", 0, 299)
    finally:
        c.stop()


def test_executor_failure_retried_elsewhere():
    from idunno.runtime.executor import FakeExecutor

    class Broken(FakeExecutor):
        def run(self, *a, **k):
            raise RuntimeError("simulated HIP error")

    c = LocalCluster(num_nodes=4, executor_factory=lambda i: Broken() if i == 2 else FakeExecutor(), **FAST).start()
    try:
        cl = c.client()
        cl.inference(0, 399, "resnet18")
        s = cl.wait_idle(10, {"resnet18": 400})
        assert s["done"]["resnet18"] == 400
        check_results(cl, "resnet18", 0, 399)
    finally:
        c.stop()


def test_standby_mirrors_by_deltas(cluster):
    """After the first full snapshot the coordinator pushes only the job-table
    mutations since the standby's ack; the standby's mirror catches up."""
    coord = cluster.coordinator()
    sb = cluster.nodes[coord.standby]
    cl = cluster.client()
    cl.inference(0, 3999, "resnet18")
    cl.wait_idle(10, {"resnet18": 4000})
    synced = lambda: sb.state.mirror_seq == coord.state.seq and coord._standby_ack == (0, coord.state.seq)  # noqa: E731
    assert wait_for(synced, 5), (sb.state.mirror_seq, coord.state.seq, coord._standby_ack)
    big = coord.meta_bytes
    cl.inference(4000, 4399, "resnet18")
    cl.wait_idle(10, {"resnet18": 4400})
    assert wait_for(synced, 5)
    # one query = a few log entries; the push no longer carries the 11 earlier queries
    assert coord.meta_bytes < 8000, coord.meta_bytes
    assert sorted(q for q in sb.state.worker_set) == sorted(q for q in coord.state.worker_set)
    assert big >= 0


def test_sdfs_hbm_holders_are_version_checked(cluster):
    """a late HBM_HAS for an older version must not re-publish a
    stale HBM copy; peers are offered only holders of the current version."""
    from idunno.runtime.messages import Type

    n = cluster.nodes["node02"]
    master = cluster.coordinator()
    assert n.sdfs.put_bytes(b"x" * 64, "images/shard_0")["ver"] == 1
    n.sdfs.announce_hbm("images/shard_0", ver=1)
    assert wait_for(lambda: master.sdfs._master_locate("images/shard_0")["hbm"] == ["node02"], 2)
    assert n.sdfs.put_bytes(b"y" * 64, "images/shard_0")["ver"] == 2      # re-put clears holders
    assert master.sdfs._master_locate("images/shard_0")["hbm"] == []
    # the old announcement arrives late: recorded as version 1, never offered
    master.sdfs.handle({"t": Type.HBM_HAS, "name": "images/shard_0", "node": "node03", "held": True, "ver": 1,
                        "src": "node03"})
    assert master.sdfs._master_locate("images/shard_0")["hbm"] == []
    master.sdfs.handle({"t": Type.HBM_HAS, "name": "images/shard_0", "node": "node04", "held": True, "ver": 2,
                        "src": "node04"})
    assert master.sdfs._master_locate("images/shard_0")["hbm"] == ["node04"]
    # a holder asked for another version than it caches exports nothing
    calls = []
    n.sdfs.hbm_provider = lambda name, pid, ver: calls.append(ver)
    n.sdfs.handle({"t": Type.FETCH_HBM, "name": "images/shard_0", "pid": 1, "ver": 2, "src": "node05"})
    assert calls == [2]


def test_ipc_local_parking_expires(monkeypatch):
    """a same-process hand-off whose consumer never came is dropped
    after LOCAL_TTL_S instead of pinning the tensor forever."""
    from idunno.runtime import ipc

    class T:
        is_cuda = True
        shape = (2, 3)

        def is_contiguous(self):
            return True

    monkeypatch.setattr(ipc, "LOCAL_TTL_S", 0.05)
    import os

    meta = ipc.export_tensor(T(), consumer_pid=os.getpid())
    assert meta["local"] in ipc._LOCAL
    time.sleep(0.1)
    ipc.export_tensor(T(), consumer_pid=os.getpid())     # any export prunes expired entries
    assert meta["local"] not in ipc._LOCAL
    with pytest.raises(KeyError):
        ipc.import_copy(meta, "cuda:0")
