"""Self-validation and self-tuning of an N > 1 step before a timed run.

The one-rank-per-GPU node runs step forms that a one-GPU box can only rehearse with
ranks time-sharing the card (the one-launch tile exchange of the 2-layer DP / FSDP
step, the deep engine's in-kernel exchange, the pipeline's stream and sync
schedules).  Before anything is timed, ``bench.py`` therefore

* **validates** every candidate form against the plain collective form: each is built
  from the same seed, runs ``k`` eager steps of the real batch with AdamW(eps = 10) --
  an update proportional to the gradient, so a wrong tile is not hidden by Adam's
  normalisation -- and its fp32 masters and first / second moments are compared with
  the reference form's, globally and per 16 x 16 block of the largest weight, and
  (DP) bit for bit across ranks.  A candidate that times out or disagrees is dropped on
  every rank and the reason is recorded;
* **tunes**: the surviving candidates are captured like the timed run and replayed in
  alternation; the fastest (max over ranks) is the one the timed run uses.

The table goes into the bench JSON (``details.autotune``).  Reference semantics being
protected: the DP step's pmean of the gradients (/root/reference/data_paral.py:210-228)
and the FSDP reduce-scatter-mean (/root/reference/param_sharding.py:129-142).
"""
from __future__ import annotations

import contextlib
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from ..runtime import dist as D

# validation bounds (relative L2 errors vs the reference form after k steps; measured on
# the shared-GPU rehearsal at W = 2, profiles/r5_autotune_validation.txt session 12: 4e-8 to
# 7e-4 whole-tensor, <= 3e-3 per block -- fp32 summation order only)
REL_TOL = 1e-2          # whole master delta / m / v
BLOCK_TOL = 0.05        # worst 16 x 16 block of the largest weight's master delta
VALIDATE_STEPS = 3
PROBE_EPS = 10.0
CONTAMINATION = 1.10    # reference re-timed after a state-changing candidate: slower by > 10 %


@dataclass
class Candidate:
    name: str
    env: Dict[str, str]
    reference: bool = False          # the plain-collective form the others are checked against
    replicated: bool = False         # the masters are replicated (DP): bit-identical across ranks
    args: Dict = field(default_factory=dict)   # bench argument overrides (PP microbatches ...)
    # trainer attribute telling whether the form this candidate asks for actually engaged
    engaged: Callable = field(default=lambda tr: True)
    # replicated over a sub-group only (hybrid DP x PP: the data axis of each stage);
    # group_of(tr) -> process group, None = the world
    group_of: Optional[Callable] = None
    # building it may change process state for everything built after it (a schedule on
    # concurrent streams opens extra hardware queues that the process keeps: round 5,
    # GPipe-8 1.9 -> 90 ms per step after a stage-streams candidate was built).  Such
    # candidates are validated and timed LAST, the reference form is re-timed after them,
    # and the table says "contaminated" when it slowed by more than CONTAMINATION
    contaminates: bool = False


@contextlib.contextmanager
def env_override(kv: Dict[str, str]):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _sync(dev):
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize(dev)


def close_trainer(tr):
    if tr is not None and hasattr(tr, "close"):
        tr.close()


def _all(flag: bool, dev) -> bool:
    """AND over the world (collective)."""
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev if D.backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def _max(v: float, dev) -> float:
    t = torch.tensor([float(v)], dtype=torch.float64, device=dev if D.backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def snapshot(tr) -> Dict[str, torch.Tensor]:
    """fp32 masters / m / v of this rank's optimizer state (FSDP: its shards)."""
    P, o = tr.state.params, tr.state.opt_state
    n = P.numel
    out = {"p": P.master[:n].detach().clone()}
    for k in ("m", "v"):
        if isinstance(o, dict) and k in o and torch.is_tensor(o[k]):
            out[k] = o[k][:n].detach().clone()
    w = max(P.names(), key=lambda nm: P.p(nm).numel())
    out["_w"] = (P.offsets[w][0], tuple(P.p(w).shape))
    return out


def _rel(a: torch.Tensor, b: torch.Tensor) -> float:
    d = float(torch.linalg.vector_norm((a - b).double()))
    r = float(torch.linalg.vector_norm(b.double()))
    return d / r if r > 0 else (0.0 if d == 0 else float("inf"))


def _block_rel(a: torch.Tensor, b: torch.Tensor, bs: int = 16) -> float:
    """Worst relative L2 error over bs x bs blocks (rows / cols zero-padded)."""
    R, Cc = a.shape
    pr, pc = (-R) % bs, (-Cc) % bs
    d = torch.nn.functional.pad((a - b).double(), (0, pc, 0, pr))
    r = torch.nn.functional.pad(b.double(), (0, pc, 0, pr))
    shp = (d.shape[0] // bs, bs, d.shape[1] // bs, bs)
    dn = d.reshape(shp).pow(2).sum(dim=(1, 3)).sqrt()
    rn = r.reshape(shp).pow(2).sum(dim=(1, 3)).sqrt()
    # blocks whose reference update is below the fp32 resolution of the masters are noise
    floor = 1e-6 * float(rn.max()) + 1e-30
    live = rn > floor
    if not bool(live.any()):
        return 0.0
    return float((dn[live] / rn[live]).max())


def compare(init: Dict, got: Dict, ref: Dict) -> Dict[str, float]:
    """Relative errors of a candidate's state against the reference form's, both after
    the same steps from ``init``."""
    out = {"p": _rel(got["p"] - init["p"], ref["p"] - init["p"])}
    for k in ("m", "v"):
        if k in got and k in ref:
            out[k] = _rel(got[k], ref[k])
    off, shp = ref["_w"]
    n = 1
    for s in shp:
        n *= s
    if len(shp) == 2:
        dg = (got["p"] - init["p"])[off:off + n].view(shp)
        dr = (ref["p"] - init["p"])[off:off + n].view(shp)
        out["block"] = _block_rel(dg, dr)
    return out


def replicated_bitwise(t: torch.Tensor, dev, group=None) -> bool:
    """``t`` identical on every rank of ``group`` (default: the world), elementwise
    MAX == MIN; the verdict is agreed over the world (collective on every rank)."""
    on = dev if D.backend() == "nccl" else "cpu"
    hi, lo = t.to(on).clone(), t.to(on).clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    return _all(bool(torch.equal(hi, lo)), dev)


def step_error(tr) -> Optional[str]:
    """This rank's in-kernel error words after eager steps (synchronises)."""
    eng = getattr(tr, "fused", None)
    tx = getattr(eng, "tx", None)
    if tx is not None and tx.error():
        return "tile exchange wait timed out"
    zt = getattr(eng, "ztick", None)
    if zt is not None and getattr(eng, "ahead_ok", False) and int(zt[1].item()) != 0:
        return f"run-ahead error word {int(zt[1].item())}"
    for xg in (getattr(tr, "xg", None), getattr(getattr(tr, "sp", None), "xg", None)):
        if xg is not None and xg.error():
            return "xgmi collective timed out"
    p2p = getattr(tr, "p2p", None)
    if p2p is not None and p2p.error():
        return "pipeline receive timed out"
    pk = getattr(tr, "pp_kernel", None)
    if pk is not None and pk.error():
        return "pipeline stage kernel wait timed out"
    return None


def _first_reason(err: Optional[str]) -> str:
    """The lowest failing rank's error text, on every rank (collective)."""
    errs = [None] * D.world_size()
    dist.all_gather_object(errs, err)
    return next((f"rank {r}: {e}" for r, e in enumerate(errs) if e), "unknown")


def _inject_corruption(tr):
    """Rehearsal hook (JDT_BENCH_FAKE_TX_CORRUPT=<rank>): on this rank one 16 x 16 block
    of the candidate's largest weight moves by 1e-3 (~1000x its 3-step update) -- what a
    mis-summed or mis-owned exchange tile looks like after the steps."""
    P = tr.state.params
    w = max(P.names(), key=lambda nm: P.p(nm).numel())
    v = P.p(w)
    if v.dim() == 2:
        blk = v[:16, :16]
        blk.add_(blk.sign() * 1e-3)
    else:
        v[:16].add_(1e-3)


def time_candidate(tr, batch, steps: int, dev) -> float:
    """us per step (max over ranks) of ``steps`` captured steps."""
    _sync(dev)
    D.barrier()
    t0 = time.perf_counter()
    if hasattr(tr, "run_steps"):
        tr.run_steps(batch, steps)
    else:
        for _ in range(steps):
            tr.step(batch)
    _sync(dev)
    dt = time.perf_counter() - t0
    return _max(dt / steps * 1e6, dev)


def _validate(c: Candidate, build: Callable, dev, validate: bool, ref: Optional[Dict], row: Dict,
              prepare_probe: Optional[Callable] = None):
    """Build ``c`` under its env, run the probe steps and fill ``row`` (valid / engaged /
    err / reason).  Returns this candidate's (init, state) snapshots (the reference form's
    become ``ref``).  ``prepare_probe(tr, batch)`` (optional) captures the trainer after
    its first eager step so the remaining probe steps run as ONE multi-step replay -- the
    form the timed run replays (a persistent multi-step launch is then validated itself,
    not only its one-step sibling); it returns False when there is nothing to capture."""
    if not validate:   # timing only (the in-kernel error words are still checked)
        row["valid"] = True
        return None
    # the env stays in force through the eager steps: engines are built (and read their
    # switches) on the first step, not at construction
    with env_override(c.env):
        tr, batch = build(PROBE_EPS, c)
        try:
            init = snapshot(tr)
            tr.step(batch)
            if prepare_probe is not None and hasattr(tr, "run_steps") and prepare_probe(tr, batch):
                tr.run_steps(batch, VALIDATE_STEPS - 1)
            else:
                for _ in range(VALIDATE_STEPS - 1):
                    tr.step(batch)
            _sync(dev)
            # the form asked for must have engaged on every rank (its engine is built on
            # the first step); otherwise it is the reference form under another name
            eng = _all(bool(c.engaged(tr)), dev)
            row["engaged"] = eng
            err = step_error(tr)
            if err is None and not c.reference and os.environ.get("JDT_BENCH_FAKE_TX_ERROR", "-1") == str(D.rank()):
                err = "tile exchange wait timed out (injected: JDT_BENCH_FAKE_TX_ERROR)"
            if not _all(err is None, dev):
                row["valid"] = False
                row["reason"] = _first_reason(err)
                return None
            if not eng and not c.reference:
                row["valid"] = None
                row["reason"] = "not engaged (the trainer fell back to the reference form)"
                return None
            if os.environ.get("JDT_BENCH_FAKE_TX_CORRUPT", "-1") == str(D.rank()) and not c.reference:
                _inject_corruption(tr)
            got = snapshot(tr)
            if c.reference:
                row["valid"] = True
            else:
                e = compare(ref["init"], got, ref["got"])
                worst = {k: _max(v, dev) for k, v in e.items()}
                row["err"] = {k: float(f"{v:.3g}") for k, v in worst.items()}
                ok = all(worst[k] <= REL_TOL for k in ("p", "m", "v") if k in worst)
                ok = ok and worst.get("block", 0.0) <= BLOCK_TOL
                row["valid"] = _all(ok, dev)
                if not row["valid"]:
                    row["reason"] = "state differs from the reference form"
            if row["valid"] and c.replicated and not c.reference:
                # DP (or a hybrid's data axis): the masters are replicated -- bit-identical
                grp = c.group_of(tr) if c.group_of is not None else None
                rep = replicated_bitwise(got["p"], dev, grp)
                row["replicated"] = rep
                if not rep:
                    row["valid"] = False
                    row["reason"] = "masters not bit-identical across the replicas"
            return {"init": init, "got": got}
        finally:
            close_trainer(tr)


def _build_timed(c: Candidate, build: Callable, prepare: Callable, steps: int):
    with env_override(c.env):
        tr, batch = build(None, c)
        for _ in range(2):
            tr.step(batch)
        prepare(tr, batch)
        tr.run_steps(batch, min(steps, 20)) if hasattr(tr, "run_steps") else tr.step(batch)
    return tr, batch


def run(cands: List[Candidate], build: Callable, prepare: Callable, dev, validate: bool = True,
        steps: int = 100, rounds: int = 3, log: Callable = print, prepare_probe: Optional[Callable] = None):
    """Validate and time ``cands`` (collective: every rank calls it with the same list).

    ``build(eps, cand)`` builds a trainer and its batch under the current env (eps: AdamW
    eps override, None = the run's own; ``cand.args``: argument overrides);
    ``prepare(tr, batch)`` captures it the way the timed run will.  Returns (report,
    trainer, batch): the report {"candidates": [...], "choice": name, "env": {...},
    "args": {...}} and the winner's trainer -- built with the run's own optimizer,
    stepped, captured and replayed, ready for the timed run (None if no candidate could
    be timed, or the reference form itself failed: the caller then builds the reference
    form itself).

    Candidates marked ``contaminates`` go last: validated and built after every other
    candidate was timed, then timed in alternation with all of them again; if the
    reference form is more than CONTAMINATION slower in that second phase the report
    says so, and the choice uses the second phase's times (the process the timed run
    will use is the contaminated one)."""
    table = []
    ref_snap = None
    order = sorted(cands, key=lambda c: (c.contaminates, not c.reference))   # reference first
    rows = {}
    for c in order:
        row = {"name": c.name, "env": dict(c.env)}
        if c.args:
            row["args"] = dict(c.args)
        table.append(row)
        rows[c.name] = row
    ref_c = next((c for c in order if c.reference), order[0])

    def no_choice(reason):
        return ({"candidates": table, "choice": ref_c.name, "env": dict(ref_c.env), "args": dict(ref_c.args),
                 "reason": reason}, None, None)

    early = [c for c in order if not c.contaminates]
    late = [c for c in order if c.contaminates]
    live = []
    for c in early:
        snap = _validate(c, build, dev, validate, ref_snap, rows[c.name], prepare_probe)
        if c.reference:
            ref_snap = snap
            if validate and not rows[c.name]["valid"]:
                # nothing to compare against: validate nothing, time nothing
                for c2 in order:
                    if c2 is not c:
                        rows[c2.name]["valid"] = None
                        rows[c2.name]["reason"] = "not validated (the reference form failed)"
                return no_choice(f"reference form failed: {rows[c.name].get('reason')}")
        if rows[c.name]["valid"]:
            live.append(c)
    built = []
    times: Dict[str, List[float]] = {}
    after: Dict[str, List[float]] = {}
    keep = None
    contaminated = False
    try:
        for c in live:
            tr, batch = _build_timed(c, build, prepare, steps)
            built.append((c, tr, batch))
        times = {c.name: [] for c, _, _ in built}
        for _ in range(rounds if len(built) > 1 else 1):
            for c, tr, batch in built:
                times[c.name].append(time_candidate(tr, batch, steps, dev))
        late_live = []
        for c in late:
            _validate(c, build, dev, validate, ref_snap, rows[c.name], prepare_probe)
            if rows[c.name]["valid"]:
                late_live.append(c)
        if late_live:
            for c in late_live:
                tr, batch = _build_timed(c, build, prepare, steps)
                built.append((c, tr, batch))
            after = {c.name: [] for c, _, _ in built}
            for _ in range(rounds):
                for c, tr, batch in built:
                    after[c.name].append(time_candidate(tr, batch, steps, dev))
            if ref_c.name in times and times[ref_c.name]:
                pre, post = min(times[ref_c.name]), min(after[ref_c.name])
                contaminated = post > CONTAMINATION * pre
                rows[ref_c.name]["us_per_step_after_late"] = round(post, 2)
        for c, tr, _ in built:
            err = step_error(tr)
            if not _all(err is None, dev):
                times[c.name] = after[c.name] = [float("inf")]
                rows[c.name]["valid"] = False
                rows[c.name]["reason"] = f"timed replays: {_first_reason(err)}"
        use = after if contaminated else {**{k: v for k, v in times.items()}, **{k: v for k, v in after.items()
                                                                                 if k not in times}}
        for c, _, _ in built:
            r = rows[c.name]
            if c.name in times:
                r["us_per_step"] = round(min(times[c.name]), 2)
            if c.name in after:
                r["us_per_step" if c.name not in times else "us_per_step_late_phase"] = round(min(after[c.name]), 2)
        ok = [(c, min(use[c.name])) for c, _, _ in built if c.name in use and min(use[c.name]) != float("inf")]
        if ok:
            best = min(ok, key=lambda x: x[1])[0]
            keep = next(x for x in built if x[0] is best)
    finally:
        for b in built:
            if b is not keep:
                close_trainer(b[1])
    if keep is None:
        return no_choice("no candidate timed")
    summary = ", ".join(f"{r['name']}: {r.get('us_per_step')}" for r in table)
    log(f"[autotune] {summary} -> {keep[0].name}" + (" (reference slowed after a late candidate)" if contaminated
                                                      else ""))
    out = {"candidates": table, "choice": keep[0].name, "env": dict(keep[0].env), "args": dict(keep[0].args),
           "steps_timed": steps, "rounds": rounds}
    if late:
        out["contaminated"] = contaminated
    return out, keep[1], keep[2]
