"""ISA check (CPU: hipcc cross-compiles gfx950): the hot fused-MLP backward kernels and
the one-launch exchange compile without readfirstlane waterfall loops -- every buffer
resource they build is wave-uniform (tools/isa_waterfalls.py; md_bwd's wave index and
step parity through readfirstlane, common.h sys_rsrc_u; the FSDP one-launch variant's
partial stores through one uniform resource per candidate owner)."""
import pathlib
import shutil
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

pytestmark = [pytest.mark.slow,
              pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not available")]

CSRC = ROOT / "jax_distributed_tuts_amd" / "ops" / "csrc"


@pytest.mark.parametrize("src", ["mlp_deep.hip", "mlp_fused.hip"])
def test_backward_kernels_have_no_waterfall_loops(src):
    from isa_waterfalls import count

    cnt = count(CSRC / src)
    assert cnt, "no kernels found"
    bad = {k: v for k, v in cnt.items() if v}
    assert not bad, bad
