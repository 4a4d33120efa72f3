"""bench.py's recovery from a one-launch N > 1 step whose in-kernel tile exchange fails
after its start-up self-test passed (bench.one_launch_failed): every rank agrees, rebuilds
on the three-launch step and still reports a measurement (the driver's scaling run must
not lose a point to it).  Rehearsed with 2 ranks sharing the GPU and a rank that reports
a failure (JDT_BENCH_FAKE_TX_ERROR); the plain run is the control."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _bench(strategy, fake):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update({"JDT_BACKEND": "gloo", "PYTHONPATH": ROOT})
    env.pop("JDT_BENCH_FAKE_TX_ERROR", None)
    if fake is not None:
        env["JDT_BENCH_FAKE_TX_ERROR"] = str(fake)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--strategy", strategy, "--steps", "20",
                        "--warmup", "5", "--no-comm-sweep"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=200)
    assert r.returncode == 0, r.stdout[-1500:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("strategy", ["dp", "fsdp"])
def test_bench_falls_back_when_the_exchange_fails(strategy):
    ok = _bench(strategy, None)
    assert "one_launch_fallback" not in ok["config"]
    assert ok["config"]["step_launches"].startswith("1 (run-ahead mlp2_bwd")
    j = _bench(strategy, 1)
    assert "one_launch_fallback" in j["config"], j["config"]
    assert not j["config"].get("step_launches", "").startswith("1 "), j["config"]
    assert j["value"] > 0 and j["n_gpus"] == 2
