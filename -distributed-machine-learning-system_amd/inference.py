"""Single-process inference entry point — the reference's L4 API
``deeplearning(filename, modelname, start_image, end_image)``
(alexnet_resnet.py:12-92) re-built on resident models.

    results, seconds = deeplearning("resnet18", "resnet18", 0, 399)
    # results: [("test_0.JPEG", "<category>", prob), ...]  (end inclusive)

Differences from the reference, all deliberate:
  * the model is built once per (model, device) and cached, not re-loaded from
    torch.hub on every call (A6); weights are random-init (no network);
  * images ``./<filename>/test_<i>.JPEG`` are decoded in memory and never
    rewritten on disk (A14); when the directory does not exist the
    deterministic synthetic 224x224x3 dataset of the cluster is used instead;
  * the chunk runs as batched forwards of ``batch`` images (``batch=1`` keeps
    the reference's one-image-at-a-time behaviour) — on the HIP kernels when a
    GPU is present, else on the fp32 PyTorch modules (CPU plumbing path,
    BASELINE.json config 1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import torch

from .models.reference import canonical
from .runtime.data import JpegSource, SyntheticSource
from .runtime.executor import HipExecutor, TorchExecutor
from .runtime.jobstate import class_names

_EXECUTORS: dict = {}
_LOCK = threading.Lock()


def _executor(device: torch.device, seed: int):
    key = (str(device), seed)
    with _LOCK:
        ex = _EXECUTORS.get(key)
        if ex is None:
            ex = HipExecutor(device, seed=seed) if device.type == "cuda" else TorchExecutor(device, seed=seed)
            _EXECUTORS[key] = ex
    return ex


def deeplearning(filename: str, modelname: str, start_image: int, end_image: int, *,
                 device: str | torch.device | None = None, batch: int | None = None, seed: int = 0,
                 data_seed: int = 1234, root: str = "."):
    """Classify images ``start_image..end_image`` (inclusive).  Returns
    ``(list[(image_name, category, prob)], elapsed_seconds)`` like the reference."""
    t0 = time.time()
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    device = torch.device(device)
    model = canonical(modelname)
    ex = _executor(device, seed)
    d = os.path.join(root, filename)
    src = JpegSource(device, root=d) if os.path.isdir(d) else SyntheticSource(data_seed, device)
    names = class_names()
    n = end_image - start_image + 1
    batch = n if not batch or batch <= 0 else batch
    out = []
    for s in range(start_image, end_image + 1, batch):
        e = min(s + batch - 1, end_image)
        cls, prob = ex.run(model, src.get(s, e), s, e)
        out += [(f"test_{s + i}.JPEG", names[int(c)], float(p)) for i, (c, p) in enumerate(zip(cls, prob))]
    return out, time.time() - t0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="one-process inference over test_<i>.JPEG (or synthetic) images")
    ap.add_argument("model", help="alexnet | resnet18 | resnet | resnet34 | resnet50")
    ap.add_argument("start", type=int)
    ap.add_argument("end", type=int)
    ap.add_argument("--dir", default=None, help="image directory (default: ./<model>, else synthetic)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--batch", type=int, default=0, help="images per forward (1 = reference behaviour)")
    a = ap.parse_args(argv)
    res, dt = deeplearning(a.dir or a.model, a.model, a.start, a.end, device=a.device, batch=a.batch)
    for r in res:
        print(json.dumps(r))
    print(f"{len(res)} images in {dt:.3f} s ({len(res) / max(dt, 1e-9):.1f} img/s)", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
