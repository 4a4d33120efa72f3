"""CPU checks of bench.py's self-validation / self-tuning driver (utils/autotune.py) on a
stand-in trainer whose step form is picked from the environment when its engine is
built -- on the FIRST step, as the real trainers do (the one-launch DP / FSDP engines,
the deep exchanges, the GPipe stage kernel).  One gloo rank."""
import os

import pytest
import torch
import torch.distributed as dist

from jax_distributed_tuts_amd.utils import autotune as AT

FORM = "JDT_TEST_FORM"


class _Flat:
    def __init__(self):
        self.master = torch.linspace(-1.0, 1.0, 32 * 32)
        self.numel = self.master.numel()
        self.offsets = {"w": (0, (32, 32))}

    def names(self):
        return ["w"]

    def p(self, name):
        return self.master.view(32, 32)


class _State:
    def __init__(self):
        self.params = _Flat()
        self.opt_state = {"m": torch.zeros(32 * 32), "v": torch.zeros(32 * 32)}


class _Trainer:
    """form "one" / "ref": the same update; "bad": a wrong 16 x 16 block."""

    def __init__(self, eps):
        self.state, self.form, self.eps, self.closed = _State(), None, eps, False

    def step(self, batch):
        if self.form is None:   # engine built on the first step, from the env of that moment
            self.form = os.environ.get(FORM, "ref")
        g = torch.cos(self.state.params.master)
        if self.form == "bad":
            g.view(32, 32)[:16, :16] += 1.0
        o = self.state.opt_state
        o["m"].mul_(0.9).add_(0.1 * g)
        o["v"].mul_(0.999).add_(0.001 * g * g)
        self.state.params.master.sub_(1e-3 * g)

    def run_steps(self, batch, n):
        for _ in range(n):
            self.step(batch)

    def close(self):
        self.closed = True


@pytest.fixture(scope="module")
def gloo1():
    if not dist.is_initialized():
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:29671", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def _cands(other):
    return [AT.Candidate("ref", {FORM: "ref"}, reference=True),
            AT.Candidate(other, {FORM: other}, engaged=lambda tr: tr.form == other)]


def _build(eps, c):
    return _Trainer(eps), None


def test_candidate_env_reaches_the_first_step(gloo1):
    # the engine of each candidate is built under that candidate's env (the bug this
    # pins: validating both forms under the caller's env compared a form with itself)
    report, tr, _ = AT.run(_cands("one"), _build, lambda tr, b: None, torch.device("cpu"), steps=2, rounds=1,
                           log=lambda *a: None)
    rows = {r["name"]: r for r in report["candidates"]}
    assert rows["one"]["engaged"] is True and rows["one"]["valid"] is True, rows
    assert rows["one"]["err"]["p"] == 0.0
    assert tr is not None and tr.form == report["choice"]
    assert FORM not in os.environ


def test_wrong_tile_is_rejected(gloo1):
    report, tr, _ = AT.run(_cands("bad"), _build, lambda tr, b: None, torch.device("cpu"), steps=2, rounds=1,
                           log=lambda *a: None)
    rows = {r["name"]: r for r in report["candidates"]}
    assert rows["bad"]["engaged"] is True
    assert rows["bad"]["valid"] is False and "differs" in rows["bad"]["reason"], rows
    assert report["choice"] == "ref" and tr.form == "ref"


def test_failed_reference_validates_nothing(gloo1):
    # the reference form's probe fails (an in-kernel wait timed out): no candidate can be
    # compared -- none is timed, the caller builds the reference form itself
    class _Bad(_Trainer):
        def __init__(self, eps):
            super().__init__(eps)
            self.fused = type("E", (), {"tx": type("T", (), {"error": lambda self: 1})()})()

    report, tr, _ = AT.run(_cands("one"), lambda eps, c: (_Bad(eps), None), lambda tr, b: None,
                           torch.device("cpu"), steps=2, rounds=1, log=lambda *a: None)
    rows = {r["name"]: r for r in report["candidates"]}
    assert tr is None and report["choice"] == "ref" and "reference form failed" in report["reason"]
    assert rows["ref"]["valid"] is False and rows["one"]["valid"] is None, rows


def test_state_changing_candidate_is_timed_last(gloo1):
    # a candidate that slows the process for everything built after it: validated and
    # timed after the others, the reference re-timed, the slowdown reported
    import time

    slow = {"on": False}

    class _T(_Trainer):
        def step(self, batch):
            super().step(batch)
            if slow["on"]:
                time.sleep(2e-3)

    order = []

    def build(eps, c):
        order.append(c.name)
        if c.name == "streams" and eps is None:
            slow["on"] = True
        return _T(eps), None

    cands = [AT.Candidate("streams", {FORM: "one"}, contaminates=True),
             AT.Candidate("ref", {FORM: "ref"}, reference=True),
             AT.Candidate("other", {FORM: "one"})]
    report, tr, _ = AT.run(cands, build, lambda tr, b: None, torch.device("cpu"), steps=3, rounds=1,
                           log=lambda *a: None)
    assert order[-1] == "streams" and order[:4] == ["ref", "other", "ref", "other"], order
    assert report["contaminated"] is True, report
    rows = {r["name"]: r for r in report["candidates"]}
    assert rows["ref"]["us_per_step_after_late"] > rows["ref"]["us_per_step"]
    slow["on"] = False


def test_probe_runs_the_captured_multi_step_form(gloo1):
    # a form that is right step by step but wrong in its captured multi-step replay (as a
    # persistent multi-step launch could be): the probe captures after the first eager
    # step and replays the rest, so the wrong replay is what gets validated -- and rejected
    class _Replay(_Trainer):
        captured = False

        def run_steps(self, batch, n):
            for _ in range(n):
                self.step(batch)
                if self.captured and self.form == "bad-replay":
                    self.state.params.master.view(32, 32)[:16, :16] += 1e-3

    def prep(tr, b):
        tr.captured = True
        return True

    cands = [AT.Candidate("ref", {FORM: "ref"}, reference=True),
             AT.Candidate("bad-replay", {FORM: "bad-replay"}, engaged=lambda tr: tr.form == "bad-replay")]
    report, tr, _ = AT.run(cands, lambda eps, c: (_Replay(eps), None), lambda tr, b: None, torch.device("cpu"),
                           steps=2, rounds=1, log=lambda *a: None, prepare_probe=prep)
    rows = {r["name"]: r for r in report["candidates"]}
    assert rows["bad-replay"]["valid"] is False and "differs" in rows["bad-replay"]["reason"], rows
    assert report["choice"] == "ref"
