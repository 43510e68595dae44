"""GPU-to-GPU tensor hand-off between two node processes (runtime/ipc.py):
a child process exports a HIP IPC handle for an HBM tensor, this process maps
it and copies it (on a 1-GPU box both processes share the device; on a node
the copy crosses xGMI)."""
import base64
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import base64, json, sys
import torch
from idunno.runtime.ipc import export_tensor
n = int(sys.argv[1])
t = (torch.arange(n, device="cuda", dtype=torch.int64) * 7 % 251).to(torch.uint8)
t2 = t[n // 2:]                          # a view with a storage offset
meta = [export_tensor(t), export_tensor(t2.contiguous())]
for m in meta:
    for k, v in list(m.items()):
        if isinstance(v, bytes):
            m[k] = {"b64": base64.b64encode(v).decode()}
print(json.dumps(meta), flush=True)
sys.stdin.readline()                      # keep the allocations alive until the parent is done
"""


def _decode(m):
    return {k: (base64.b64decode(v["b64"]) if isinstance(v, dict) else v) for k, v in m.items()}


def test_ipc_copy_between_processes():
    from idunno.runtime.ipc import import_copy

    n = 75 * (1 << 20) + 12345
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-c", CHILD, str(n)], cwd=ROOT, env=env, stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline()
        assert line, p.stderr.read()
        meta = [_decode(m) for m in json.loads(line)]
        want = (torch.arange(n, device="cuda", dtype=torch.int64) * 7 % 251).to(torch.uint8)
        got = import_copy(meta[0], "cuda")
        assert got.shape == (n,) and torch.equal(got, want)
        out = torch.empty(n - n // 2, dtype=torch.uint8, device="cuda")
        got2 = import_copy(meta[1], "cuda", out=out)
        assert got2.data_ptr() == out.data_ptr() and torch.equal(got2, want[n // 2:])
    finally:
        p.stdin.write("done\n")
        p.stdin.flush()
        p.wait(60)
    assert p.returncode == 0, p.stderr.read()
