"""__graft_entry__.smoke() on the GPU: passes on the real kernels and FAILS when the
persistent headline replay runs on a stale hand-off (JDT_SMOKE_INJECT=stale-logits: the
primed graph replayed although nothing ran the first step's forward)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _smoke(inject=None):
    env = {k: v for k, v in os.environ.items() if k != "JDT_SMOKE_INJECT"}
    env["PYTHONPATH"] = ROOT
    if inject:
        env["JDT_SMOKE_INJECT"] = inject
    return subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.smoke()"], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=300)


def test_smoke_passes_and_checks_the_persistent_kernel():
    r = _smoke()
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "persistent 4-step launch vs 4 one-step launches" in r.stdout, r.stdout


def test_smoke_fails_on_stale_logits():
    r = _smoke("stale-logits")
    assert r.returncode != 0, r.stdout
    assert "persistent vs per-step launches" in r.stderr, r.stderr[-3000:]
