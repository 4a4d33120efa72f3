"""bench.py's protection of the driver's N > 1 run (utils/autotune.py, bench.run_autotune
and bench.one_launch_failed): before the timed region every rank validates the one-launch
step (in-kernel tile exchange) against the three-launch step from the same init and
drops it -- on every rank, with the reason in the JSON -- when a wait times out OR when
its state is wrong; the surviving forms are timed and the fastest runs.  Rehearsed with
2 ranks sharing the GPU: a rank that reports a failed exchange (JDT_BENCH_FAKE_TX_ERROR),
a rank whose one-launch state is corrupted by one 16 x 16 block
(JDT_BENCH_FAKE_TX_CORRUPT), and the plain run as the control."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _bench(strategy, fake=None, corrupt=None, extra=()):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update({"JDT_BACKEND": "gloo", "PYTHONPATH": ROOT})
    for k in ("JDT_BENCH_FAKE_TX_ERROR", "JDT_BENCH_FAKE_TX_CORRUPT"):
        env.pop(k, None)
    if fake is not None:
        env["JDT_BENCH_FAKE_TX_ERROR"] = str(fake)
    if corrupt is not None:
        env["JDT_BENCH_FAKE_TX_CORRUPT"] = str(corrupt)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--strategy", strategy, "--steps", "20",
                        "--warmup", "5", "--no-comm-sweep", *extra], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=200)
    assert r.returncode == 0, r.stdout[-1500:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def _rows(j):
    return {r["name"]: r for st in j["details"]["autotune"]["stages"] for r in st["candidates"]}


@pytest.mark.parametrize("strategy", ["dp", "fsdp"])
def test_autotune_validates_and_falls_back(strategy):
    ok = _bench(strategy)
    rows = _rows(ok)
    assert rows["one-launch"]["valid"] is True and rows["one-launch"]["engaged"] is True, rows
    assert rows["three-launch"]["valid"] is True, rows
    assert all(r["us_per_step"] > 0 for r in rows.values()), rows
    print(strategy, "errors of the one-launch form vs three-launch:", rows["one-launch"]["err"])
    # N > 1 persistent launch (the exchange inside every step): validated like the others
    assert rows["persistent"]["valid"] is True and rows["persistent"]["engaged"] is True, rows
    print("errors of the persistent form vs three-launch:", rows["persistent"]["err"])
    if strategy == "dp":
        assert rows["one-launch"]["replicated"] is True
        assert rows["persistent"]["replicated"] is True
    # the timed run is the faster valid form
    best = min(rows.values(), key=lambda r: r["us_per_step"])["name"]
    assert ok["details"]["autotune"]["stages"][0]["choice"] == best
    sl = ok["config"].get("step_launches", "")
    assert sl.startswith("1 (run-ahead mlp2_bwd") == (best == "one-launch"), ok["config"]
    assert sl.startswith("1/") == (best == "persistent"), ok["config"]
    assert "one_launch_fallback" not in ok["config"]
    # a corrupted exchange tile on rank 1: wrong values, not a timeout -> dropped everywhere
    j = _bench(strategy, corrupt=1)
    rows = _rows(j)
    assert rows["one-launch"]["valid"] is False and "differs" in rows["one-launch"]["reason"], rows
    assert rows["one-launch"]["err"]["block"] > 0.05, rows
    assert rows["persistent"]["valid"] is False and "differs" in rows["persistent"]["reason"], rows
    assert "one_launch_fallback" in j["config"], j["config"]
    assert not j["config"].get("step_launches", "").startswith(("1 ", "1/")), j["config"]
    assert j["value"] > 0 and j["n_gpus"] == 2
    # a failed exchange wait reported by rank 1
    j = _bench(strategy, fake=1)
    rows = _rows(j)
    assert rows["one-launch"]["valid"] is False and "timed out" in rows["one-launch"]["reason"], rows
    assert not j["config"].get("step_launches", "").startswith(("1 ", "1/")), j["config"]


@pytest.mark.parametrize("strategy", ["dp", "fsdp"])
def test_bench_falls_back_when_the_exchange_fails_without_autotune(strategy):
    ok = _bench(strategy, extra=("--autotune", "off"))
    assert "one_launch_fallback" not in ok["config"]
    # a 20-step replay is one persistent launch per rank (JDT_DP_PST / JDT_FSDP_PST default on)
    want = "1/20 (persistent"
    assert ok["config"]["step_launches"].startswith(want), ok["config"]
    j = _bench(strategy, 1, extra=("--autotune", "off"))
    assert "one_launch_fallback" in j["config"], j["config"]
    assert not j["config"].get("step_launches", "").startswith(("1 ", "1/")), j["config"]
    assert j["value"] > 0 and j["n_gpus"] == 2


def test_pp_autotune_validates_the_stage_kernel():
    """GPipe with one layer per stage (2 ranks sharing the GPU): the autotune value-checks
    the in-kernel stage step against the per-tick launches (AdamW eps = 10 probe, no
    dropout) before timing it, and drops it -- reason in the JSON -- when one rank's
    stage state is corrupted by one 16 x 16 block."""
    extra = ("--hidden-layers", "2")
    ok = _bench("pp", extra=extra)
    rows = _rows(ok)
    assert rows["stage-kernel=1"]["valid"] is True and rows["stage-kernel=1"]["engaged"] is True, rows
    assert rows["stage-kernel=1"]["err"]["p"] < 1e-2, rows
    assert all(r["valid"] for r in rows.values()), rows
    assert "pp_rejected" not in ok["config"]
    j = _bench("pp", corrupt=1, extra=extra)
    rows = _rows(j)
    assert rows["stage-kernel=1"]["valid"] is False and "differs" in rows["stage-kernel=1"]["reason"], rows
    assert "stage-kernel=1" in j["config"]["pp_rejected"], j["config"]
    assert j["details"]["autotune"]["stages"][-1]["choice"] == "stage-kernel=0"
    assert "step_launches" not in j["config"], j["config"]   # the per-tick path ran
    assert j["value"] > 0 and j["n_gpus"] == 2
