"""Native host-side checks under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5.2): csrc/tests/host_checks.cpp exercises the kernels' own
__host__ __device__ index math (csrc/tile_math.h: XCD remap bijectivity, LDS
swizzle permutations and bank-conflict freedom).  Host code only: GPU sanitizers
are not available on the GPU pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "-distributed-machine-learning-system_amd", "csrc", "tests", "host_checks.cpp")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_host_index_math_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_checks"
    cmd = [HIPCC, "--offload-host-only", "-O1", "-g", "-std=c++17",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=all", SRC, "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s)" in r.stdout
