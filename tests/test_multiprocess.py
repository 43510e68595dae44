"""Real multi-process cluster on localhost TCP (one OS process per node, as on
an MI355X host), fake executor on the CPU.  Nodes are SIGKILLed mid-query to
exercise failure detection, chunk re-dispatch and standby promotion across
process boundaries (SURVEY.md §4 "multi-process single node")."""
import ast
import os
import signal
import socket
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ephemeral_low() -> int:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            return int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        return 32768


def _base_port(n):
    """n consecutive free ports BELOW the ephemeral range: a range taken from
    the ephemeral ports races the outgoing connections other tests (and other
    processes) open meanwhile ("Address already in use")."""
    import random

    hi = max(_ephemeral_low() - n - 1, 11000)
    for _ in range(50):
        p = random.randint(10000, hi)
        ok = True
        for i in range(n):
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", p + i))
            except OSError:
                ok = False
            finally:
                t.close()
        if ok:
            return p
    raise RuntimeError("no port range")


def wait_listening(ports, timeout: float = 60.0, procs=None) -> None:
    """Block until every port accepts a TCP connection (a started node's
    control plane is up) instead of sleeping a fixed time: a loaded machine
    can take seconds to import torch in each child."""
    end = time.monotonic() + timeout
    left = set(ports)
    while left:
        for p in list(left):
            try:
                socket.create_connection(("127.0.0.1", p), timeout=0.2).close()
                left.discard(p)
            except OSError:
                pass
        if left:
            if procs and any(pr.poll() is not None for pr in procs):
                raise RuntimeError("a node process exited during start-up")
            if time.monotonic() > end:
                raise TimeoutError(f"ports {sorted(left)} not listening after {timeout}s")
            time.sleep(0.05)


@pytest.mark.slow
def test_multiprocess_cluster_failures():
    n = 4
    base = _base_port(n)
    tmp = tempfile.mkdtemp(prefix="idunno_mp_")
    env = dict(os.environ, IDUNNO_HEARTBEAT_PERIOD_S="0.05", IDUNNO_FAILURE_TIMEOUT_S="0.6",
               IDUNNO_METADATA_PERIOD_S="0.1", PYTHONPATH=ROOT)
    procs = {}
    for i in range(n - 1):
        procs[i] = subprocess.Popen(
            [sys.executable, "-m", "idunno.launch", "node", "--index", str(i), "--nodes", str(n),
             "--base-port", str(base), "--store-root", tmp, "--executor", "fake", "--join-delay", "0.3"],
            cwd=ROOT, env=env, stdin=subprocess.DEVNULL, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    cfg = ClusterConfig(num_nodes=n, base_port=base, store_root=tmp, heartbeat_period_s=0.05,
                        failure_timeout_s=1.2, metadata_period_s=0.1, rpc_timeout_s=3.0)
    me = Node(cfg, "node03", TcpTransport("node03", cfg.address, cfg.address("node03")), FakeExecutor())
    try:
        wait_listening([base + i for i in range(n - 1)], procs=list(procs.values()))
        me.start(join=True)
        assert wait_for(lambda: len(me.membership.alive()) == n, 15), me.membership.table()
        cl = Client(me)
        cl.inference(0, 799, "resnet18")
        s = cl.wait_idle(20, {"resnet18": 800})
        assert s["done"]["resnet18"] == 800, s

        # slow node01 down, start a query, SIGKILL it while it holds a chunk
        assert cl.kill("node01", "delay", 1.5)
        time.sleep(0.1)
        cl.inference(800, 1199, "alexnet")
        time.sleep(0.3)
        procs[1].send_signal(signal.SIGKILL)
        s = cl.wait_idle(20, {"alexnet": 400})
        assert s["done"]["alexnet"] == 400, s

        # SIGKILL the coordinator: the standby (this process) promotes itself
        procs[0].send_signal(signal.SIGKILL)
        assert wait_for(lambda: me.is_coordinator, 10)
        cl.inference(1200, 1599, "resnet18")
        s = cl.wait_idle(20, {"resnet18": 1200})
        assert s["done"]["resnet18"] == 1200, s
        res = cl.view("c4")["results"]
        idx = set()
        for k, chunks in res.items():
            for ch in chunks:
                idx |= {int(t[0][5:-5]) for t in ast.literal_eval(ch)}
        assert idx == set(range(1600))
    finally:
        me.stop()
        for p in procs.values():
            if p.poll() is None:
                p.kill()
            p.wait(10)
