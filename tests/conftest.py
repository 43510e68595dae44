import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the HIP extension")
    config.addinivalue_line("markers", "slow: multi-second test")
    config.addinivalue_line("markers", "experimental: needs the kernels built only with IDUNNO_EXPERIMENTAL=1 "
                                       "(measured-and-dropped loops); deselected otherwise")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    # the measured-and-dropped experimental kernels are not in the default
    # _C.so: their tests are deselected (not reported as skips) unless that
    # build was asked for
    if os.environ.get("IDUNNO_EXPERIMENTAL") != "1":
        drop = [it for it in items if "experimental" in it.keywords]
        if drop:
            config.hook.pytest_deselected(items=drop)
            items[:] = [it for it in items if "experimental" not in it.keywords]
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
