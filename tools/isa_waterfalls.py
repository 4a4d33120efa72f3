"""Count readfirstlane "waterfall" loops per kernel in the gfx950 ISA of csrc files.

A buffer access whose resource descriptor the compiler cannot prove wave-uniform (a
pointer or size that reached it through a VGPR -- a value derived from threadIdx, loaded
by a vector load, or merged after a lane-dependent branch) is compiled into a loop that
readfirstlane's the descriptor, runs the access for the lanes that match, and repeats:
~12 extra instructions around every such access even when all lanes agree.  Round 4 found
20-58 per hot md_bwd variant and 48-54 in the one-launch exchange kernels (fixed with
readfirstlane on the wave index / step parity, common.h sys_rsrc_u).

    python tools/isa_waterfalls.py [file.hip ...]   (default: every ops/ and comm/ csrc file)
"""
from __future__ import annotations

import pathlib
import re
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "jax_distributed_tuts_amd"


def count(src: pathlib.Path) -> dict:
    with tempfile.TemporaryDirectory() as d:
        out = pathlib.Path(d) / "k.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "--cuda-device-only", "-S", str(src), f"-I{PKG / 'ops' / 'csrc'}", "-o", str(out),
                        "-Wno-pass-failed", "-Wno-unused-value"], check=True, capture_output=True)
        lines = out.read_text().split("\n")
    cur, cnt = None, {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            cur = m.group(1)
            cnt.setdefault(cur, 0)
        if cur and "Inner Loop Header" in ln and i + 1 < len(lines) and "readfirstlane" in lines[i + 1]:
            cnt[cur] += 1
    return cnt


def main(argv):
    files = [pathlib.Path(a) for a in argv] or sorted((PKG / "ops" / "csrc").glob("*.hip")) + sorted(
        (PKG / "comm" / "csrc").glob("*.hip"))
    total = 0
    for f in files:
        cnt = count(f)
        nz = {k: v for k, v in cnt.items() if v}
        total += sum(nz.values())
        print(f"{f.name}: {len(cnt)} kernels, {len(nz)} with waterfall loops")
        for k, v in sorted(nz.items(), key=lambda x: -x[1]):
            print(f"  {v:4d}  {k}")
    print(f"total waterfall loops: {total}")


if __name__ == "__main__":
    main(sys.argv[1:])
