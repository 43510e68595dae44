"""Loader for the native extension ``idunno._C``.

Policy (no silent fallbacks): if a GPU is present the HIP extension MUST
load — a missing or stale ``_C.so`` raises instead of quietly running an eager
PyTorch path.  On a CPU-only host ``available()`` is False and callers use the
torch reference executor explicitly.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _gpu_present() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def load(build_if_missing: bool | None = None):
    """Import (and, if allowed, build) the extension.  Raises on failure."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        import torch  # noqa: F401  (loads libamdhip64 / libc10 before _C)

        if build_if_missing is None:
            build_if_missing = os.environ.get("IDUNNO_AUTOBUILD", "1") == "1"
        from .. import _build

        if build_if_missing and _build.needs_build():
            _build.build()
        try:
            _mod = importlib.import_module("idunno._C")
        except Exception as e:  # noqa: BLE001
            _err = e
            raise RuntimeError(
                "idunno native extension failed to load; run `python -m idunno._build`"
            ) from e
        return _mod


def available() -> bool:
    """True when the HIP path can run (GPU present and extension loadable)."""
    if not _gpu_present():
        return False
    load()  # raises loudly on a GPU host without a working extension
    return True


def so_path() -> str:
    from .. import _build

    return str(_build.TARGET)
