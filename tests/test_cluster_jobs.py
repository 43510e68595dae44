"""Coordinator-side batching (reference two-tier variant) and
straggler resend (A7), on the in-memory fake cluster."""
from idunno.runtime.cluster import LocalCluster
from idunno.runtime.shell import Shell

FAST = dict(heartbeat_period_s=0.05, failure_timeout_s=1.0, metadata_period_s=0.1, rpc_timeout_s=2.0)


def test_job_submission_batched_by_coordinator():
    c = LocalCluster(num_nodes=4, **FAST).start()
    try:
        cl = c.client()
        sh = Shell(c.nodes["node03"], cl)
        assert sh.execute("job 0 1049 alexnet") == "coordinator batching 3 alexnet queries"
        s = cl.wait_idle(10, {"alexnet": 1050})
        assert s["done"]["alexnet"] == 1050
        assert s["finished_queries"]["alexnet"] == 3
        st = c.coordinator().state
        with st.lock:
            qs = list(st.worker_set)
        assert sorted(q for (m, q) in qs if m == "alexnet") == [1, 2, 3]
    finally:
        c.stop()


def test_job_resumed_by_promoted_standby():
    """A coordinator-side job that is still being cut into queries when the
    coordinator dies is resumed by the standby from the replicated job cursor."""
    c = LocalCluster(num_nodes=5, client_query_interval_s=0.05, **FAST).start()
    try:
        cl = c.client("node03")
        r = cl.submit_job(0, 3999, "resnet18")          # 10 queries, 50 ms apart
        assert r["queries"] == 10
        import time

        time.sleep(0.22)                                  # a few queries dispatched
        c.crash("node00")
        s = cl.wait_idle(15, {"resnet18": 4000})
        assert s["done"]["resnet18"] == 4000, s           # nothing lost, nothing double counted
        assert c.coordinator().name == "node04"
    finally:
        c.stop()


def test_job_survives_coordinator_crash_before_any_periodic_snapshot():
    """The job is replicated when it is created, not only by the periodic push
    (metadata period >> time to crash here): the promoted standby resumes it,
    re-sends chunks it has no results for, and counts every image exactly once."""
    cfg = dict(FAST, metadata_period_s=30.0)
    c = LocalCluster(num_nodes=5, client_query_interval_s=0.02, **cfg).start()
    try:
        for n in c.nodes.values():
            n.extra_delay_s = 0.05                         # chunks in flight at the crash
        cl = c.client("node03")
        r = cl.submit_job(0, 3999, "resnet18")
        assert r["queries"] == 10
        import time

        time.sleep(0.12)
        c.crash("node00")
        s = cl.wait_idle(20, {"resnet18": 4000})
        assert s["done"]["resnet18"] == 4000 and s["pending"] == 0, s
        assert c.coordinator().name == "node04"
    finally:
        c.stop()


def test_straggler_resend():
    c = LocalCluster(num_nodes=4, straggler_resend=True, straggler_timeout_s=0.3, **FAST).start()
    try:
        c.nodes["node02"].extra_delay_s = 3.0       # alive (answers pings) but very slow
        cl = c.client()
        cl.inference(0, 399, "resnet18")
        s = cl.wait_idle(2.5, {"resnet18": 400})
        assert s["done"]["resnet18"] == 400, s      # finished before the straggler would have
    finally:
        c.stop()
