"""Interactive shell — same command set as the reference (README.md:31-50,
mp4_machinelearning.py:1111-1229), plus fault-injection commands.

``Shell.execute(line) -> str`` is pure (returns the text it would print), so
every command is unit-testable; ``repl()`` wraps it around ``input()``.
"""
from __future__ import annotations

import json
import shlex

from .data import put_synthetic_dataset

MENU = """\
1. list_mem: list the membership list
2. list_self: list self's id
3. join: command to join the group
4. leave: command to voluntarily leave the group (different from a failure, which will be Ctrl-C or kill)
5. list_master: list master (coordinator) and standby
6. grep <regex>: grep every live node's log (MP1 distributed grep)
7. put localfilename sdfsfilename: upload localfilename from local dir to sdfs
8. get sdfsfilename localfilename: get file from sdfs to local
9. delete sdfsfilename: delete file from sdfs
10.ls sdfsfilename: list all nodes where this file is currently being stored
11.store: list all files currently being stored at this node
12.get-versions sdfsfilename num-versions localfilename: last num-versions versions, newest first, delimited
13.inference <start> <end> <model>: submit queries (model: alexnet | resnet18 | resnet | resnet50)
c1 query rate and finished inferences for each model
c2 current processing time of a query for each model (mean, q1, q2, q3, stddev)
c4 query results (also written to result.txt)
cvm (c5) tasks running on each node
cq how each query is distributed: (node, start, end, state, t_start, t_end)
job <start> <end> <model>: send the whole range; the coordinator cuts it into batch-size queries
dataset <n_images> [shard_images]: put a synthetic 224x224x3 dataset into SDFS
trace <file.json>: write every node's query/chunk spans as a Chrome trace
checkpoint: write the coordinator's job state to disk (restart with IDUNNO_RESUME=1)
kill-rank <node|rank> | kill-coordinator | delay-rank <node|rank> <seconds>: fault injection
  (kill / delay are aliases of kill-rank / delay-rank)
exit"""

ARITY_ERR = "Error: missing or too many {} parameter ."


class Shell:
    def __init__(self, node, client):
        self.node = node
        self.client = client

    def execute(self, line: str) -> str:
        try:
            parts = shlex.split(line.strip())
        except ValueError as e:
            return f"Error: {e}"
        if not parts:
            return ""
        cmd, args = parts[0], parts[1:]
        n = self.node

        def need(k):
            if len(args) != k:
                raise _Arity(cmd)

        try:
            if cmd in ("1", "list_mem"):
                return json.dumps(n.membership.table(), indent=1)
            if cmd in ("2", "list_self"):
                return n.membership.self_id()
            if cmd in ("3", "join"):
                return "joined" if n.membership.join() else "join failed"
            if cmd in ("4", "leave"):
                n.membership.leave()
                return "left"
            if cmd in ("5", "list_master"):
                return f"coordinator: {n.membership.master} (epoch {n.membership.epoch}); standby: {n.standby}"
            if cmd in ("6", "grep"):
                if not args:
                    raise _Arity(cmd)
                return "\n".join(self.client.grep(" ".join(args)))
            if cmd in ("7", "put"):
                need(2)
                r = n.sdfs.put(args[0], args[1])
                return f"put {args[1]} version {r.get('ver')} on {r.get('replicas')}"
            if cmd in ("8", "get"):
                need(2)
                return "ok" if n.sdfs.get(args[0], args[1]) else f"{args[0]} not found"
            if cmd in ("9", "delete"):
                need(1)
                return "deleted" if n.sdfs.delete(args[0]) else f"{args[0]} not found"
            if cmd in ("10", "ls"):
                need(1)
                return str(n.sdfs.ls(args[0]))
            if cmd in ("11", "store"):
                return str(n.sdfs.store_list())
            if cmd in ("12", "get-versions"):
                need(3)
                k = int(args[1])
                if k <= 0:
                    return "Error: num-versions must be a positive integer"
                got = n.sdfs.get_versions(args[0], k, args[2])
                return f"wrote {got} versions to {args[2]}"
            if cmd in ("13", "inference"):
                need(3)
                self.client.inference_async(int(args[0]), int(args[1]), args[2])
                return f"submitting {args[2]} queries for [{args[0]}, {args[1]}]"
            if cmd == "job":
                need(3)
                r = self.client.submit_job(int(args[0]), int(args[1]), args[2])
                return f"coordinator batching {r.get('queries')} {args[2]} queries"
            if cmd == "c4":
                res = self.client.c4("result.txt")
                return str(res)
            if cmd in ("cvm", "c5", "cq", "c1", "c2"):
                return self.client.view(cmd).get("text", "")
            if cmd == "dataset":
                if len(args) not in (1, 2):
                    raise _Arity(cmd)
                k = put_synthetic_dataset(n.sdfs, int(args[0]), n.cfg.data_seed,
                                          int(args[1]) if len(args) > 1 else 500)
                return f"put {k} shards"
            if cmd == "trace":
                need(1)
                return f"wrote {self.client.trace(args[0])} trace events to {args[0]}"
            if cmd == "checkpoint":
                return f"checkpoint written to {self.client.checkpoint().get('path')}"
            if cmd in ("kill", "kill-rank"):
                need(1)
                return "sent" if self.client.kill(self._node_arg(args[0])) else "unreachable"
            if cmd == "kill-coordinator":
                need(0)
                return "sent" if self.client.kill(n.membership.master) else "unreachable"
            if cmd in ("delay", "delay-rank"):
                need(2)
                return ("sent" if self.client.kill(self._node_arg(args[0]), "delay", float(args[1]))
                        else "unreachable")
            if cmd in ("help", "menu"):
                return MENU
            if cmd == "exit":
                return "exit"
            return "Invalid input. Please try again"
        except _Arity as e:
            return ARITY_ERR.format(e.cmd)
        except Exception as e:  # noqa: BLE001
            return f"Error: {type(e).__name__}: {e}"

    def _node_arg(self, a: str) -> str:
        """A node name, or a rank index (``kill-rank 3`` -> node03)."""
        return self.node.cfg.node_name(int(a)) if a.isdigit() else a

    def repl(self) -> None:
        print(MENU)
        while True:
            try:
                line = input("Please enter input: ")
            except EOFError:
                return
            out = self.execute(line)
            if out == "exit":
                return
            if out:
                print(out)


class _Arity(Exception):
    def __init__(self, cmd):
        self.cmd = cmd
