"""Host-side AddressSanitizer run of the kernel library's launchers:
every csrc/*.hip is rebuilt with ``-Xarch_host -fsanitize=address`` and
tools/asan_host_check.cpp drives the host code paths that need no GPU."""
import shutil
import subprocess
import sys

import pytest

pytestmark = pytest.mark.slow


@pytest.mark.skipif(shutil.which("hipcc") is None and not __import__("os").path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_asan_host_check():
    r = subprocess.run([sys.executable, "-m", "jax_distributed_tuts_amd.ops.build", "--asan-check"],
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "0 failure(s)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr
