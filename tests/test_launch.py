"""One command, N ranks: ``bench.py --gpus N`` and the entry
scripts start N local ranks themselves when no launcher did, report the real
world size, and refuse to run a job of the wrong size.  CPU: the ranks' process
group is gloo (the same code path as RCCL on a GPU node)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.slow


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "JDT_SIM_CPU")}
    env.update({"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": "", "PYTHONPATH": ROOT})
    env.update(kw)
    return env


def _run(args, env=None, timeout=300):
    return subprocess.run([sys.executable, *args], cwd=ROOT, env=env or _env(), capture_output=True, text=True,
                          timeout=timeout)


def _why(r) -> str:
    """A failed job's whole output: every rank's stderr (the ranks share the parent's
    stream), so a rank's faulthandler stack and native abort message are never cut off
    (a one-off SIGABRT of rank 1 in round 5 left only its last 3000 characters)."""
    return f"exit {r.returncode}\n--- stdout ---\n{r.stdout[-4000:]}\n--- stderr (all ranks) ---\n{r.stderr[-60000:]}"


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_bench_gpus_n_starts_n_ranks(n):
    r = _run(["bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, _why(r)
    j = _json_line(r.stdout)
    assert j["n_gpus"] == n and j["steps"] == 2 and j["warmup"] == 1
    assert j["config"]["parallelism"] == f"dp{n}"
    assert j["details"]["process_group"] == "gloo"


def test_bench_refuses_wrong_world_size():
    r = _run(["bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1"], env=_env(WORLD_SIZE="1"))
    assert r.returncode == 3
    assert "2 ranks requested" in r.stderr


@pytest.mark.parametrize("script,extra,title", [
    ("data_paral.py", [], "dp"),
    ("param_sharding.py", ["--steps", "1"], "FSDP - Final metrics"),
    ("pipeline_parallel.py", ["--hidden-layers", "2", "--dp", "1"], "PP2 x DP1 - Final metrics"),
])
def test_entry_scripts_gpus_flag(script, extra, title):
    r = _run([script, "--gpus", "2", "--steps", "1", "--check-replication", *extra])
    assert r.returncode == 0, _why(r)
    assert title in r.stdout and "loss:" in r.stdout
    assert "[check-replication]" in r.stdout


def test_local_launch_propagates_failure(tmp_path):
    """A failing rank's status becomes the job's; the other ranks are stopped
    (they would otherwise wait forever on the dead peer)."""
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(7)
        time.sleep(120)
    """))
    code = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        from jax_distributed_tuts_amd.runtime.launch import local_launch
        t = time.time()
        rc = local_launch(3, [{str(script)!r}], grace_s=5)
        print("rc", rc, "dt", round(time.time() - t))
    """)
    r = _run(["-c", code], timeout=120)
    assert r.returncode == 0, r.stderr
    rc, dt = r.stdout.split()[1], float(r.stdout.split()[3])
    assert rc == "7" and dt < 60
