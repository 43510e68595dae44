"""Span tracing (Chrome trace export) and coordinator checkpoint / resume."""
import json

from idunno.config import ClusterConfig
from idunno.runtime.cluster import LocalCluster
from idunno.runtime.shell import Shell
from idunno.runtime.transport import wait_for

FAST = dict(heartbeat_period_s=0.05, failure_timeout_s=1.0, metadata_period_s=0.1, rpc_timeout_s=2.0)


def test_chrome_trace_has_query_and_chunk_spans(tmp_path):
    c = LocalCluster(num_nodes=3, **FAST).start()
    try:
        cl = c.client()
        cl.inference(0, 199, "alexnet")
        cl.wait_idle(5, {"alexnet": 200})
        sh = Shell(c.nodes["node02"], cl)
        out = sh.execute(f"trace {tmp_path / 't.json'}")
        assert out.startswith("wrote")
        evs = json.loads((tmp_path / "t.json").read_text())["traceEvents"]
        names = {e["name"] for e in evs}
        assert {"query.submit", "chunk.stage", "chunk.compute", "result.ingest"} <= names
        assert {e["pid"] for e in evs if e["name"] == "chunk.compute"} == {"node00", "node01", "node02"}
    finally:
        c.stop()


def test_checkpoint_and_resume_after_full_restart(tmp_path):
    cfg = ClusterConfig(num_nodes=3, store_root=str(tmp_path), log_dir=str(tmp_path / "logs"), **FAST)
    c = LocalCluster(cfg).start()
    try:
        cl = c.client()
        for n in c.nodes.values():
            n.extra_delay_s = 5.0                    # nothing finishes before the "power cut"
        cl.inference(0, 299, "resnet18")
        assert wait_for(lambda: len(c.coordinator().state.pending()) == 3, 2)
        assert "checkpoint written" in Shell(c.nodes["node01"], cl).execute("checkpoint")
    finally:
        c.stop()
    # whole cluster restarts; the coordinator resumes its in-flight query from disk
    cfg2 = ClusterConfig(num_nodes=3, store_root=str(tmp_path), log_dir=str(tmp_path / "logs2"), resume=True, **FAST)
    c2 = LocalCluster(cfg2).start()
    try:
        cl2 = c2.client()
        s = cl2.wait_idle(10, {"resnet18": 300})
        assert s["done"]["resnet18"] == 300
        st = c2.coordinator().state
        with st.lock:
            assert st.next_qnum["resnet18"] == 1   # same query, not re-submitted
    finally:
        c2.stop()
