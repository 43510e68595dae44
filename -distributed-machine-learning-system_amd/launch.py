"""Process launcher: one node process per GPU on one MI355X host.

  python -m idunno.launch node --index I [--shell] [--executor hip|torch|fake]
        run node I (TCP control plane on base_port + I, GPU I % ngpu)
  python -m idunno.launch cluster --nodes N [--shell-node K]
        spawn N node processes as children; node K (default N-1) runs in the
        foreground with the interactive shell (reference: every VM runs
        ``python3 mp4_machinelearning.py`` and gets the REPL, README.md:26)

Config comes from ``--config file.{json,yaml}``, IDUNNO_* env vars and flags
(see ``idunno.config``).  Children are started with ``subprocess`` — never
``exec`` — so no GPU context is ever replaced in place.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import threading
import time


def _cfg(a):
    from .config import ClusterConfig

    over = {"num_nodes": a.nodes, "base_port": a.base_port, "store_root": a.store_root,
            "log_dir": a.log_dir, "coordinator": a.coordinator, "standby": a.standby}
    return ClusterConfig.load(a.config, **{k: v for k, v in over.items() if v is not None})


def run_node(a) -> int:
    import logging

    import torch

    from .runtime.client import Client
    from .runtime.data import SdfsSource, SyntheticSource
    from .runtime.executor import make_executor
    from .runtime.node import Node
    from .runtime.shell import Shell
    from .runtime.transport import TcpTransport

    logging.basicConfig(level=logging.WARNING, format="%(asctime)s %(name)s %(message)s")
    cfg = _cfg(a)
    name = cfg.node_name(a.index)
    if torch.cuda.is_available() and a.executor in ("auto", "hip"):
        dev = torch.device("cuda", a.index % torch.cuda.device_count())
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    ex = make_executor(a.executor, dev if dev.type == "cuda" else None, seed=cfg.model_seed, dtype=cfg.dtype,
                       fp32_impl=cfg.fp32_impl)
    if cfg.collective_rounds is None:
        # one node per process and per GPU: queries run as RCCL rounds by default
        # (RCCL needs a distinct GPU per rank; nodes sharing a GPU use the TCP path)
        cfg.collective_rounds = dev.type == "cuda" and a.executor in ("auto", "hip") and \
            torch.cuda.device_count() >= cfg.num_nodes      # (a single node: one-member rounds)
    tr = TcpTransport(name, cfg.address, cfg.address(name))
    node = Node(cfg, name, tr, ex)
    node.source = (SdfsSource(node.sdfs, dev, peer_copy=cfg.sdfs_peer_copy) if a.source == "sdfs"
                   else SyntheticSource(cfg.data_seed, dev))
    if a.index != cfg.coordinator:
        time.sleep(a.join_delay)
    node.start(join=True)
    if a.shell:
        Shell(node, Client(node)).repl()
        node.stop()
        return 0
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    while not stop.wait(0.5) and node.alive_flag:
        pass
    node.stop()
    return 0


def run_cluster(a) -> int:
    cfg = _cfg(a)
    shell_node = cfg.num_nodes - 1 if a.shell_node is None else a.shell_node
    procs = []
    base = [sys.executable, "-m", "idunno.launch", "node", "--executor", a.executor, "--source", a.source]
    for flag, v in (("--config", a.config), ("--nodes", cfg.num_nodes), ("--base-port", cfg.base_port),
                    ("--store-root", cfg.store_root), ("--log-dir", a.log_dir)):
        if v is not None:
            base += [flag, str(v)]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for i in range(cfg.num_nodes):
        if i == shell_node and not a.no_shell:
            continue
        procs.append(subprocess.Popen(base + ["--index", str(i)], env=env, stdin=subprocess.DEVNULL))
    rc = 0
    try:
        if not a.no_shell:
            a2 = argparse.Namespace(**vars(a))
            a2.index, a2.shell = shell_node, True
            rc = run_node(a2)
        else:
            for p in procs:
                p.wait()
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("mode", choices=["node", "cluster"])
    ap.add_argument("--index", type=int, default=0)
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--config", default=None)
    ap.add_argument("--base-port", type=int, default=None)
    ap.add_argument("--store-root", default=None)
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--coordinator", type=int, default=None)
    ap.add_argument("--standby", type=int, default=None)
    ap.add_argument("--executor", default="auto", choices=["auto", "hip", "torch", "fake"])
    ap.add_argument("--source", default="synthetic", choices=["synthetic", "sdfs"])
    ap.add_argument("--shell", action="store_true")
    ap.add_argument("--shell-node", type=int, default=None)
    ap.add_argument("--no-shell", action="store_true")
    ap.add_argument("--join-delay", type=float, default=0.5)
    a = ap.parse_args(argv)
    return run_node(a) if a.mode == "node" else run_cluster(a)


if __name__ == "__main__":
    sys.exit(main())
