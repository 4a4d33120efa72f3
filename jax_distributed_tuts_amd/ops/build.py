"""In-tree build of the gfx950 kernel library (``ops/lib/libjdt_kernels.so``).

Every ``csrc/*.hip`` (and ``*.cpp``) file, plus ``comm/csrc/*.hip``, is compiled with
``hipcc --offload-arch=gfx950 -O3`` into an object and linked into one shared
library.  No PyTorch headers are involved: the kernels expose plain
``extern "C"`` launchers that take raw device pointers plus a ``hipStream_t``,
which ``ops/_lib.py`` calls through ctypes on torch's current stream, so the
launches are capturable into hipGraphs.  The library lives inside the package
directory so it travels with the repo snapshot to the GPU box.

Usage: ``python -m jax_distributed_tuts_amd.ops.build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
COMM_CSRC = HERE.parent / "comm" / "csrc"   # xGMI P2P collectives, linked into the same library
LIBDIR = HERE / "lib"
OBJDIR = LIBDIR / "obj"
LIB = LIBDIR / "libjdt_kernels.so"
ARCH = os.environ.get("JDT_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the kernel library)")


def sources() -> list[Path]:
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")) + list(COMM_CSRC.glob("*.hip")))


def _headers_mtime() -> float:
    hs = list(CSRC.glob("*.h")) + list(COMM_CSRC.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, force: bool) -> Path:
    obj = OBJDIR / (src.stem + ".o")
    if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _headers_mtime()):
        return obj
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", str(src), "-o", str(obj),
           "-Wno-pass-failed", "-Wno-unused-result", f"-I{CSRC}"]
    if src.suffix == ".cpp":
        cmd[1:1] = ["-x", "hip"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-4000:]}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    OBJDIR.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    jobs = jobs or min(8, max(1, len(srcs)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if force or not LIB.exists() or LIB.stat().st_mtime < newest:
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[jdt] built {LIB} from {len(objs)} sources", file=sys.stderr)
    return LIB


def is_stale() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    return any(s.stat().st_mtime > t for s in sources()) or _headers_mtime() > t


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs)
