"""Collective query rounds in the multi-process node runtime (gloo on the CPU,
the same code path that runs over RCCL with one node process per GPU).

Queries run as broadcast+gather rounds on an epoch-versioned process group;
SIGKILLing a member mid-round must fall back to TCP JOBs and re-form the group
over the survivors, and SIGKILLing the coordinator must let the promoted
standby re-form and keep serving rounds.

Liveness comes from the failure detector, not the collective timeout: the
killed member's round must be recovered within failure_timeout_s + 1 s, and an
idle gap longer than collective_timeout_s (now only the rendezvous timeout)
must not break the epoch."""
import ast
import os
import signal
import subprocess
import sys
import tempfile
import time

import pytest

from idunno.config import ClusterConfig
from idunno.runtime.client import Client
from idunno.runtime.executor import FakeExecutor
from idunno.runtime.node import Node
from idunno.runtime.transport import TcpTransport, wait_for

from test_multiprocess import ROOT, _base_port, wait_listening


def _indices(cl):
    idx = set()
    for _k, chunks in cl.view("c4")["results"].items():
        for ch in chunks:
            idx |= {int(t[0][5:-5]) for t in ast.literal_eval(ch)}
    return idx


@pytest.mark.slow
def test_collective_rounds_with_failures():
    n = 4
    base = _base_port(n)
    tmp = tempfile.mkdtemp(prefix="idunno_cr_")
    knobs = dict(IDUNNO_HEARTBEAT_PERIOD_S="0.05", IDUNNO_FAILURE_TIMEOUT_S="0.6",
                 IDUNNO_METADATA_PERIOD_S="0.1", IDUNNO_COLLECTIVE_ROUNDS="1",
                 IDUNNO_COLLECTIVE_TIMEOUT_S="2")
    env = dict(os.environ, PYTHONPATH=ROOT, **knobs)
    procs = {}
    for i in range(n - 1):
        procs[i] = subprocess.Popen(
            [sys.executable, "-m", "idunno.launch", "node", "--index", str(i), "--nodes", str(n),
             "--base-port", str(base), "--store-root", tmp, "--executor", "fake", "--join-delay", "0.3"],
            cwd=ROOT, env=env, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    cfg = ClusterConfig.load(env=knobs, num_nodes=n, base_port=base, store_root=tmp, rpc_timeout_s=3.0)
    assert cfg.collective_rounds
    me = Node(cfg, "node03", TcpTransport("node03", cfg.address, cfg.address("node03")), FakeExecutor())
    try:
        wait_listening([base + i for i in range(n - 1)], procs=list(procs.values()))
        me.start(join=True)
        assert wait_for(lambda: len(me.membership.alive()) == n, 15), me.membership.table()
        # the coordinator forms the group over all 4 nodes; this node is a member
        assert wait_for(lambda: me.rounds.group.formed and len(me.rounds.group.members) == n, 20)
        cl = Client(me)
        for q in range(3):
            cl.inference(q * 400, q * 400 + 399, "resnet18")
        s = cl.wait_idle(20, {"resnet18": 1200})
        assert s["done"]["resnet18"] == 1200, s
        assert me.rounds.rounds_done >= 3              # served as collective rounds, not TCP JOBs
        # this node is the standby: every round is gathered to it as well (second root),
        # so it holds the results itself instead of waiting for a mirror from rank 0
        assert me.name == me.standby and me.rounds.group.standby_rank == me.rounds.group.rank
        assert wait_for(lambda: me.rounds.standby_rounds >= 3, 5), me.rounds.standby_rounds

        # idle for longer than the collective timeout: the epoch survives, rounds go on
        time.sleep(3.0)
        before = me.rounds.rounds_done
        epoch = me.rounds.group.epoch
        cl.inference(1200, 1599, "resnet18")
        s = cl.wait_idle(20, {"resnet18": 1600})
        assert s["done"]["resnet18"] == 1600, s
        assert me.rounds.rounds_done > before and me.rounds.group.epoch == epoch

        # slow node01 so a round is in flight, then SIGKILL it: TCP fallback + re-form over 3
        assert cl.kill("node01", "delay", 1.5)
        time.sleep(0.1)
        cl.inference(1200, 1599, "alexnet")
        time.sleep(0.5)
        procs[1].send_signal(signal.SIGKILL)
        t_kill = time.monotonic()
        s = cl.wait_idle(30, {"alexnet": 400})
        recovered = time.monotonic() - t_kill
        assert s["done"]["alexnet"] == 400, s
        assert recovered <= cfg.failure_timeout_s + 1.0, f"dead-member round took {recovered:.2f}s"
        assert wait_for(lambda: me.rounds.group.formed and len(me.rounds.group.members) == n - 1, 30)
        before = me.rounds.rounds_done
        cl.inference(1600, 1999, "resnet18")
        s = cl.wait_idle(20, {"resnet18": 2000})
        assert s["done"]["resnet18"] == 2000, s
        assert me.rounds.rounds_done > before

        # a round the standby gathered itself survives the coordinator's death: once
        # it holds the query, SIGKILL the coordinator; the query is not run again
        sr = me.rounds.standby_rounds
        cl.inference(2400, 2799, "alexnet")
        assert wait_for(lambda: me.state.images_done("alexnet") >= 800, 10)
        assert wait_for(lambda: me.rounds.standby_rounds > sr, 5)

        # SIGKILL the coordinator: this standby promotes itself and re-forms as rank 0
        procs[0].send_signal(signal.SIGKILL)
        assert wait_for(lambda: me.is_coordinator, 10)
        # the promoted coordinator's epoch is formed and healthy (no re-form still
        # pending from the failure detector) before the next query is timed
        assert wait_for(lambda: me.rounds.group.formed and me.rounds.group.rank == 0
                        and len(me.rounds.group.members) == 2 and me.rounds.healthy, 30)
        before = me.rounds.rounds_done
        cl.inference(2000, 2399, "resnet18")
        s = cl.wait_idle(20, {"resnet18": 2400})
        assert s["done"]["resnet18"] == 2400, s
        assert me.rounds.rounds_done > before
        assert _indices(cl) == set(range(2800))
        assert me.state.images_done("alexnet") == 800
    finally:
        me.stop()
        for p in procs.values():
            if p.poll() is None:
                p.kill()
            p.wait(10)
