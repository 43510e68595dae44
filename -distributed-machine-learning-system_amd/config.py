"""Typed cluster configuration (reference C1 constants at
mp4_machinelearning.py:28-60 and utils.py:57-92).

The reference hard-codes ports by OS user, host names / IPs, batch sizes,
heartbeat periods and fixed sleeps in module constants.  Here every knob is a
dataclass field with the reference value as default where it has one, loaded
from (in increasing priority) defaults < a JSON/YAML file < IDUNNO_* env vars
< CLI flags.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field


@dataclass
class ClusterConfig:
    # -- topology: one node (rank) per GPU on one MI355X host ------------------
    num_nodes: int = 8
    host: str = "127.0.0.1"
    base_port: int = 18335                   # node i listens on base_port + i
    coordinator: int = 0                     # index of the coordinator node
    standby: int = -1                        # hot-standby node (-1 = last node)
    node_prefix: str = "node"

    # -- inference ------------------------------------------------------------
    batch_size: dict = field(default_factory=lambda: {"alexnet": 500, "resnet18": 400,
                                                      "resnet50": 1024, "resnet34": 400})
    worker_budget: int = 8                   # reference RATE_FACTOR (:44) -> GPUs shared by jobs
    max_chunk: int = 1024                    # largest per-worker batch (HBM is not the limit)
    dataset_size: int = 10000                # reference dataset: 10,000 images (report p.1)
    dtype: str = "fp32"                      # executor precision: "fp32" (the reference's) | "fp16"
    fp32_impl: str = "split"                 # fp32 kernels: "split" (split-fp16, fp32-accurate) | "f32mfma"
    prefetch: bool = True                    # stage the next queued chunk while one computes
    quick_start_wait_s: float = 0.005        # worker: wait this long for a just-queued prefetch before
                                             # answering the finished chunk first
    model_seed: int = 0
    data_seed: int = 1234

    # -- membership / failure detector ----------------------------------------
    heartbeat_period_s: float = 0.3          # reference PING period (:219)
    failure_timeout_s: float = 2.0           # reference LEAVE threshold (:847)
    metadata_period_s: float = 1.0           # reference METADATA push period (:987)
    straggler_timeout_s: float = 30.0        # reference (disabled) resend rule (:822), fixed (A7)
    straggler_resend: bool = False

    # -- pacing (reference sleeps; 0 in throughput mode) -------------------------
    client_query_interval_s: float = 0.0     # reference 20 s between queries (:1109)
    worker_start_delay_s: float = 0.0        # reference 3 s before each chunk (:594)

    # -- SDFS ---------------------------------------------------------------------
    replication: int = 4                     # reference places 4-5 replicas (utils.py:48-55)
    sdfs_peer_copy: bool = True              # shards another node holds in HBM: GPU-to-GPU copy (IPC)
    store_root: str = "/tmp/idunno"

    # -- collective data plane (one node per process only) ----------------------
    # run queries as RCCL/gloo rounds when the group is healthy; None = auto:
    # on for GPU nodes started one per process by idunno.launch
    collective_rounds: bool | None = None
    collective_backend: str = ""             # "" = auto (RCCL on GPU nodes, gloo on CPU); "gloo" on GPU
                                             # tensors rehearses N nodes on fewer GPUs (bench --rehearse-gloo)
    collective_port_offset: int = 500        # TCPStore port = base_port + offset + epoch % 100
    collective_timeout_s: float = 30.0       # rendezvous timeout; a round's liveness comes from membership
    collective_op_timeout_s: float = 120.0   # backstop for one pending collective (process-group timeout)
    abort_join_s: float = 5.0                # how long a stopping node waits for a background epoch abort
    round_depth: int = 2                     # rounds in flight (double-buffered send / gather / host)
    job_window: int = 3                      # coordinator-side job: queries in flight before the next is cut

    # -- checkpoint / resume ----------------------------------------------------
    checkpoint_period_s: float = 0.0         # coordinator writes state to disk (0 = off)
    resume: bool = False                     # coordinator restarts from its checkpoint

    # -- misc -------------------------------------------------------------------
    log_dir: str = ""
    rpc_timeout_s: float = 5.0

    def node_name(self, i: int) -> str:
        return f"{self.node_prefix}{i:02d}"

    def nodes(self) -> list[str]:
        return [self.node_name(i) for i in range(self.num_nodes)]

    def node_index(self, name: str) -> int:
        return int(name[len(self.node_prefix):])

    @property
    def coordinator_name(self) -> str:
        return self.node_name(self.coordinator)

    @property
    def standby_name(self) -> str:
        s = self.standby if self.standby >= 0 else self.num_nodes - 1
        return self.node_name(s)

    def address(self, name: str) -> tuple[str, int]:
        return self.host, self.base_port + self.node_index(name)

    def batch_for(self, model: str) -> int:
        return int(self.batch_size.get(model, 400))

    # -- loading ----------------------------------------------------------------
    def update(self, **kw) -> "ClusterConfig":
        names = {f.name for f in dataclasses.fields(self)}
        for k, v in kw.items():
            if k not in names:
                raise KeyError(f"unknown config key {k!r}")
            setattr(self, k, v)
        return self

    @classmethod
    def load(cls, path: str | None = None, env: dict | None = None, **overrides) -> "ClusterConfig":
        cfg = cls()
        if path:
            with open(path) as f:
                if path.endswith((".yaml", ".yml")):
                    import yaml

                    data = yaml.safe_load(f) or {}
                else:
                    data = json.load(f)
            cfg.update(**data)
        env = os.environ if env is None else env
        types = {f.name: f.type for f in dataclasses.fields(cls)}
        for k in types:
            ev = env.get("IDUNNO_" + k.upper())
            if ev is None:
                continue
            cur = getattr(cfg, k)
            if isinstance(cur, bool) or (cur is None and k == "collective_rounds"):
                val = ev.lower() in ("1", "true", "yes")
            elif isinstance(cur, int):
                val = int(ev)
            elif isinstance(cur, float):
                val = float(ev)
            elif isinstance(cur, dict):
                val = json.loads(ev)
            else:
                val = ev
            setattr(cfg, k, val)
        cfg.update(**{k: v for k, v in overrides.items() if v is not None})
        return cfg

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)
