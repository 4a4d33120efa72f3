"""Resource check (CPU: hipcc cross-compiles gfx950): the deep backward's N > 1 exchange
(TX) variants keep the occupancy the one-launch step's co-residency rule needs
(mlp_deep.hip md_tx_fits: two sharing ranks' 512-thread grids resident together ->
4 waves per SIMD).  Round 5's AdamW-constant pin raised the top layer's TX variant to
133 VGPRs (3 waves per SIMD) and silently turned the 2-rank one-launch deep DP step
off; the pin is now kept out of the TX variants (profiles/r5_closing3_run.txt)."""
import pathlib
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "jax_distributed_tuts_amd" / "ops" / "csrc"

pytestmark = [pytest.mark.slow,
              pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not available")]

# md_bwd_kernel<K_IN, TOP, C, KC, NN, XCD, BND, AHEAD, TX, WPE, FX>
FIELDS = ("K_IN", "TOP", "C", "KC", "NN", "XCD", "BND", "AHEAD", "TX", "WPE", "FX")


def _occupancy(src: pathlib.Path) -> dict:
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                            "--cuda-device-only", "-c", str(src), f"-I{CSRC}", "-o", str(pathlib.Path(d) / "k.o"),
                            "-Rpass-analysis=kernel-resource-usage", "-Wno-pass-failed", "-Wno-unused-value"],
                           check=True, capture_output=True, text=True)
    occ, cur = {}, None
    for ln in r.stderr.split("\n"):
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = m.group(1)
        m = re.search(r"Occupancy \[waves/SIMD\]: (\d+)", ln)
        if m and cur:
            occ[cur] = int(m.group(1))
            cur = None
    return occ


def test_md_bwd_exchange_variants_keep_co_residency_occupancy():
    occ = _occupancy(CSRC / "mlp_deep.hip")
    tx = {}
    for name, o in occ.items():
        if "md_bwd_kernel" not in name:
            continue
        vals = [int(v) for _, v in re.findall(r"L([bi])(\d+)E", name)]
        if len(vals) != len(FIELDS):
            continue
        a = dict(zip(FIELDS, vals))
        if a["TX"]:
            tx[name] = (a, o)
    assert tx, "no TX variants of md_bwd found"
    low = {n: o for n, (a, o) in tx.items() if (a["WPE"] == 4 or (a["WPE"] == 1 and a["TOP"])) and o < 4}
    assert not low, low
