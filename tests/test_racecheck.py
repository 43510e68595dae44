"""The opt-in race detector (idunno/utils/racecheck.py): it must
flag an unlocked cross-thread table access and a lock-order inversion, stay quiet
on properly locked code, and the in-process cluster must run clean under it."""
import threading
from collections import defaultdict

import pytest

from idunno.utils import racecheck


@pytest.fixture
def rc():
    racecheck.enable(True)
    racecheck.clear()
    yield racecheck
    racecheck.clear()
    racecheck.enable(False)


def _run(fn, n=2):
    ths = [threading.Thread(target=fn, name=f"t{i}") for i in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()


def test_unlocked_shared_table_is_reported(rc):
    d = rc.watch(defaultdict(list), "tbl")

    def body():
        for i in range(50):
            d[i % 3].append(i)
    _run(body)
    reps = rc.reports()
    assert len(reps) == 1 and "data race on tbl" in reps[0]


def test_locked_table_and_thread_local_table_are_clean(rc):
    lk = rc.make_lock("tbl-lock")
    d = rc.watch({}, "tbl")
    mine = rc.watch([], "private")

    def body():
        for i in range(50):
            with lk:
                d[i] = d.get(i, 0) + 1
    _run(body, 4)
    for i in range(10):          # only ever touched by this thread: exclusive, never reported
        mine.append(i)
    assert rc.reports() == []
    assert d[0] == 4


def test_lockset_refinement_catches_inconsistent_locking(rc):
    a, b = rc.make_lock("a"), rc.make_lock("b")
    d = rc.watch({}, "tbl")
    with a:
        d[0] = 1                 # main thread, exclusive
    done = threading.Event()

    def t1():
        with a:
            d[1] = 1             # shared, lockset {a}
        done.set()
    th = threading.Thread(target=t1)
    th.start()
    th.join()
    assert rc.reports() == []
    with b:
        d[2] = 1                 # lockset {a} & {b} = {} -> race
    assert any("data race on tbl" in r for r in rc.reports())


def test_lock_order_inversion_is_reported(rc):
    a, b = rc.make_lock("A"), rc.make_lock("B", reentrant=True)
    with a:
        with b:
            pass
    with b:
        with b:                  # re-entry adds no edge
            with a:
                pass
    reps = rc.reports()
    assert len(reps) == 1 and "lock-order inversion" in reps[0] and "'A'" in reps[0]


def test_raise_mode(rc):
    rc.enable(True, mode="raise")
    lk = rc.make_lock("x")
    with pytest.raises(rc.RaceError):
        lk.release()


def test_cluster_runs_clean_under_racecheck(rc):
    from idunno.runtime.cluster import LocalCluster

    c = LocalCluster(num_nodes=5, heartbeat_period_s=0.05, failure_timeout_s=1.0, metadata_period_s=0.1,
                     rpc_timeout_s=2.0).start()
    try:
        cl = c.client()
        t = cl.inference_async(0, 799, "resnet18")
        cl.inference(0, 999, "alexnet")
        t.join()
        s = cl.wait_idle(20, {"resnet18": 800, "alexnet": 1000})
        assert s["done"] == {"resnet18": 800, "alexnet": 1000}
        c.nodes["node02"].extra_delay_s = 0.5
        t = cl.inference_async(800, 1199, "resnet18")
        import time
        time.sleep(0.1)
        c.crash("node02")
        t.join()
        s = cl.wait_idle(20, {"resnet18": 1200})
        assert s["done"]["resnet18"] == 1200
    finally:
        c.stop()
    assert rc.reports() == [], "\n".join(rc.reports())
