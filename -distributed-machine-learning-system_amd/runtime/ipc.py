"""GPU-to-GPU tensor hand-off between node processes of one host (SURVEY.md
§2.5 M4: "cross-GPU replica copies ... over xGMI").

A node that holds an SDFS shard in HBM exports a HIP IPC handle for it
(``export_tensor``: the dmabuf-backed handle PyTorch's CUDA-IPC sharing
uses, HSA_ENABLE_IPC_MODE_LEGACY=0); a peer process maps the allocation and
copies it into its own HBM with one device-to-device copy
(``import_copy``) -- over xGMI when the two processes drive different GPUs,
an HBM-local copy when they share one.  The handle travels as a plain dict of
ints / bytes over the msgpack control plane; nothing is pickled.

The exporter's storage stays alive while a mapping is open: PyTorch's IPC
sent-data ref counter (ref_counter_handle / offset) delays the producer-side
free until every consumer has released its mapping, which ``import_copy``
does before it returns.
"""
from __future__ import annotations

import itertools
import os
import threading
import time

import torch

_DTYPES = {"uint8": torch.uint8, "float32": torch.float32, "float16": torch.float16, "int32": torch.int32}


# same-process hand-offs (nodes of an in-process cluster share one address
# space, and a process cannot open its own IPC handle): the tensor itself
_LOCAL: dict[int, tuple[float, torch.Tensor]] = {}
_LOCAL_LOCK = threading.Lock()
_KEYS = itertools.count(1)
# a parked tensor whose consumer never came (lost FETCH_HBM reply, timed-out
# request) is released after this long (it pinned tens of MB of HBM)
LOCAL_TTL_S = 30.0
LOCAL_MAX = 64


def _prune_locked(now: float) -> None:
    for k in [k for k, (t0, _) in _LOCAL.items() if now - t0 > LOCAL_TTL_S]:
        del _LOCAL[k]
    while len(_LOCAL) > LOCAL_MAX:
        del _LOCAL[min(_LOCAL)]


def export_tensor(t: torch.Tensor, consumer_pid: int | None = None) -> dict:
    """IPC description of a contiguous CUDA tensor (plain msgpack-able types).
    For a consumer in this same process the tensor is parked in a registry
    instead (``import_copy`` takes it from there)."""
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("export_tensor takes a contiguous CUDA tensor")
    if consumer_pid is not None and consumer_pid == os.getpid():
        key = next(_KEYS)
        now = time.monotonic()
        with _LOCAL_LOCK:
            _prune_locked(now)
            _LOCAL[key] = (now, t)
        return {"pid": os.getpid(), "local": key, "shape": list(t.shape)}
    dt = next((k for k, v in _DTYPES.items() if v == t.dtype), None)
    if dt is None:
        raise ValueError(f"unsupported dtype {t.dtype}")
    st = t.untyped_storage()
    (device, handle, size_b, off_b, rc_handle, rc_off, ev_handle, ev_sync) = st._share_cuda_()
    return {"pid": os.getpid(), "device": int(device), "handle": bytes(handle), "size_b": int(size_b), "off_b": int(off_b),
            "rc_handle": bytes(rc_handle), "rc_off": int(rc_off),
            "ev_handle": bytes(ev_handle) if ev_handle is not None else b"", "ev_sync": bool(ev_sync),
            "shape": list(t.shape), "offset": int(t.storage_offset()), "dtype": dt}


def import_copy(meta: dict, device: torch.device | int | str, out: torch.Tensor | None = None) -> torch.Tensor:
    """Map an exported tensor and copy it into a tensor on ``device``
    (``out`` if given).  Returns the copy; the mapping is closed again."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("import_copy needs a CUDA device")
    if "local" in meta:
        with _LOCAL_LOCK:
            ent = _LOCAL.pop(meta["local"], None)
        if ent is None:
            raise KeyError("parked tensor expired before it was fetched")
        src = ent[1]
        dst = out if out is not None else torch.empty_like(src, device=dev)
        dst.copy_(src, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        return dst
    dtype = _DTYPES[meta["dtype"]]
    with torch.cuda.device(dev):
        torch.cuda._lazy_init()
        storage = torch.UntypedStorage._new_shared_cuda(
            meta["device"], meta["handle"], meta["size_b"], meta["off_b"], meta["rc_handle"], meta["rc_off"],
            meta["ev_handle"] or None, meta["ev_sync"])
        src = torch.empty(0, dtype=dtype, device=storage.device).set_(
            storage, meta["offset"], tuple(meta["shape"]))
        dst = out if out is not None else torch.empty(tuple(meta["shape"]), dtype=dtype, device=dev)
        dst.copy_(src, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()      # copy done before the mapping goes away
        del src
        del storage
    return dst
