"""In-tree builder for the native extension ``idunno._C`` (gfx950 only).

Drives ``hipcc --offload-arch=gfx950`` directly (no hipify, no
torch.utils.cpp_extension JIT cache): every ``csrc/**/*.hip`` / ``*.cpp`` is
compiled to an object under ``build/`` and linked into ``_C.so`` next to this
file, so the built library travels with the repository snapshot to the GPU box.

Usage: ``python -m idunno._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD = PKG_DIR.parent / "build" / "idunno_C"
TARGET = PKG_DIR / "_C.so"
ARCH = "gfx950"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the ROCm toolchain is required to build idunno._C")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    incs = ce.include_paths(device_type="cuda")
    torch_lib = str(Path(torch.__file__).resolve().parent / "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, torch_lib, abi



def sources() -> list[Path]:
    # csrc/tests/ holds standalone host programs (sanitizer checks), not extension code
    skip = {"tests"}
    return sorted(p for p in [*CSRC.rglob("*.hip"), *CSRC.rglob("*.cpp")]
                  if not skip & set(p.relative_to(CSRC).parts))


def headers() -> list[Path]:
    return sorted(CSRC.rglob("*.h"))


def _compile_cmd(src: Path, obj: Path, incs, abi) -> list[str]:
    cmd = [
        _hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-Wno-unused-result", "-Wno-deprecated-declarations",
        f"-I{sysconfig.get_paths()['include']}", f"-I{CSRC}",
    ]
    cmd += [f"-I{i}" for i in incs]
    cmd += ["-c", str(src), "-o", str(obj)]
    return cmd


# next to the .so (not under build/, which never ships to the GPU box): a box
# that receives a prebuilt _C.so must not rebuild it for want of this file
FLAGS = PKG_DIR / "_C.so.flags"


def _flags() -> str:
    return f"arch={ARCH}"


def needs_build(force: bool = False) -> bool:
    if force or not TARGET.exists():
        return True
    if not FLAGS.exists() or FLAGS.read_text() != _flags():
        return True
    t = TARGET.stat().st_mtime
    return any(p.stat().st_mtime > t for p in [*sources(), *headers(), Path(__file__)])


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    """Compile and link ``_C.so``; returns its path.  Raises on any failure."""
    if not needs_build(force):
        return TARGET
    incs, torch_lib, abi = _torch_paths()
    BUILD.mkdir(parents=True, exist_ok=True)
    if not FLAGS.exists() or FLAGS.read_text() != _flags():
        force = True                       # a build-flag change recompiles everything
    hdr_mtime = max([p.stat().st_mtime for p in headers()] + [Path(__file__).stat().st_mtime])
    objs, todo = [], []
    for src in sources():
        obj = BUILD / (src.relative_to(CSRC).as_posix().replace("/", "__") + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_mtime):
            todo.append((src, obj))
    jobs = jobs or min(8, os.cpu_count() or 4, max(1, len(todo)))

    def run(item):
        src, obj = item
        cmd = _compile_cmd(src, obj, incs, abi)
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stdout}\n{r.stderr}")
        return src.name

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for name in ex.map(run, todo):
            if verbose:
                print(f"  compiled {name}", flush=True)
    link = [
        _hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(TARGET) + ".tmp",
        *map(str, objs), f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
        "-ltorch_hip", "-ltorch_python", f"-Wl,-rpath,{torch_lib}",
    ]
    r = subprocess.run(link, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    _check_undefined(Path(str(TARGET) + ".tmp"))
    os.replace(str(TARGET) + ".tmp", TARGET)
    FLAGS.write_text(_flags())
    return TARGET


def _check_undefined(so: Path) -> None:
    """Refuse a library that references one of its own symbols without
    defining it (e.g. a kernel launch stub the host pass silently dropped)."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    r = subprocess.run([nm, "-D", "--undefined-only", str(so)], capture_output=True, text=True)
    bad = [ln.split()[-1] for ln in r.stdout.splitlines() if "idunno" in ln]
    if bad:
        so.unlink(missing_ok=True)
        raise RuntimeError(f"link left {len(bad)} undefined idunno symbols, e.g. {bad[:3]}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(f"built {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
