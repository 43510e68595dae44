"""In-process cluster harness: N nodes on an in-memory or TCP transport.

Used by the fake multi-node tests and by ``idunno.launch
--inproc``.  Every node gets its own executor and data source (one per GPU
when several are visible; all on one device or CPU otherwise).
"""
from __future__ import annotations

import shutil
import tempfile
import time

from ..config import ClusterConfig
from .client import Client
from .node import Node
from .transport import InMemoryNetwork, TcpTransport, wait_for


class LocalCluster:
    def __init__(self, cfg: ClusterConfig | None = None, executor_factory=None, source_factory=None,
                 transport: str = "memory", net: InMemoryNetwork | None = None, **cfg_kw):
        self.tmp = None
        if cfg is None:
            self.tmp = tempfile.mkdtemp(prefix="idunno_")
            cfg = ClusterConfig(store_root=self.tmp, log_dir=self.tmp + "/logs", **cfg_kw)
        self.cfg = cfg
        self.kind = transport
        self.net = net or (InMemoryNetwork() if transport == "memory" else None)
        from .executor import FakeExecutor

        self.executor_factory = executor_factory or (lambda i: FakeExecutor())
        self.source_factory = source_factory or (lambda i, node: None)
        self.nodes: dict[str, Node] = {}

    def _transport(self, name):
        if self.kind == "memory":
            return self.net.transport(name)
        return TcpTransport(name, self.cfg.address, self.cfg.address(name))

    def make_node(self, i: int) -> Node:
        name = self.cfg.node_name(i)
        n = Node(self.cfg, name, self._transport(name), self.executor_factory(i))
        n.source = self.source_factory(i, n)
        self.nodes[name] = n
        return n

    def start(self, timeout: float = 5.0) -> "LocalCluster":
        order = [self.cfg.coordinator] + [i for i in range(self.cfg.num_nodes) if i != self.cfg.coordinator]
        for i in order:
            self.make_node(i).start(join=True)
        coord = self.nodes[self.cfg.coordinator_name]
        wait_for(lambda: len(coord.membership.alive()) == self.cfg.num_nodes, timeout)
        return self

    def client(self, name: str | None = None) -> Client:
        return Client(self.nodes[name or self.cfg.node_name(self.cfg.num_nodes - 1)])

    def coordinator(self) -> Node:
        for n in self.nodes.values():
            if n.alive_flag and n.is_coordinator:
                return n
        raise RuntimeError("no live coordinator")

    def crash(self, name: str) -> None:
        if self.kind == "memory":
            self.net.crash(name)
        self.nodes[name].stop()

    def restart(self, name: str) -> Node:
        i = self.cfg.node_index(name)
        n = self.make_node(i)
        n.membership.master = self.coordinator().name
        n.membership.epoch = self.coordinator().membership.epoch
        n.start(join=True)
        return n

    def stop(self) -> None:
        for n in self.nodes.values():
            if n.alive_flag:
                n.stop()
        if self.tmp:
            time.sleep(0.05)
            shutil.rmtree(self.tmp, ignore_errors=True)

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()
