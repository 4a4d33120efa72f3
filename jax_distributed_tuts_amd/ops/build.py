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


ASAN_OBJDIR = LIBDIR / "obj_asan"
ASAN_BIN = LIBDIR / "asan_host_check"
ASAN_DRIVER = HERE.parent.parent / "tools" / "asan_host_check.cpp"
ASAN_FLAGS = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-g"]


def asan_check(jobs: int | None = None) -> int:
    """Host-side AddressSanitizer build of every kernel source + tools/asan_host_check.cpp,
    then run it on the CPU.  Device code is compiled as usual: only the
    host part of each translation unit is instrumented.  Returns the exit status."""
    ASAN_OBJDIR.mkdir(parents=True, exist_ok=True)

    def comp(src: Path) -> Path:
        obj = ASAN_OBJDIR / (src.stem + ".o")
        if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _headers_mtime()):
            return obj
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O1", "-std=c++17", "-fPIC", "-c", str(src), "-o", str(obj),
               "-Wno-pass-failed", "-Wno-unused-result", f"-I{CSRC}", *ASAN_FLAGS]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"asan hipcc failed for {src.name}:\n{r.stderr[-4000:]}")
        return obj

    srcs = [s for s in sources() if s.suffix == ".hip"]
    with cf.ThreadPoolExecutor(jobs or min(8, len(srcs))) as ex:
        objs = list(ex.map(comp, srcs))
    drv = ASAN_OBJDIR / "asan_host_check.o"
    cmd = [_hipcc(), "-O1", "-std=c++17", "-c", str(ASAN_DRIVER), "-o", str(drv), *ASAN_FLAGS]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"asan driver compile failed:\n{r.stderr[-4000:]}")
    cmd = [_hipcc(), f"--offload-arch={ARCH}", str(drv), *map(str, objs), "-o", str(ASAN_BIN), *ASAN_FLAGS]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"asan link failed:\n{r.stderr[-4000:]}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([str(ASAN_BIN)], capture_output=True, text=True, env=env)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr[-4000:])
    return r.returncode


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--asan-check", action="store_true",
                    help="build the host-side ASan variant + tools/asan_host_check.cpp and run it on the CPU")
    a = ap.parse_args()
    if a.asan_check:
        sys.exit(asan_check(a.jobs))
    build(force=a.force, jobs=a.jobs)
