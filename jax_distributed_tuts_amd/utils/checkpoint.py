"""Checkpoint / resume (the reference has none).

Rank-local files: each rank writes ``<dir>/rank<r>.safetensors`` with its flat
fp32 master, AdamW moments, device step counter and running metrics, plus a
JSON manifest of the named views (name -> offset, local shape, global shape,
sharding names) so FSDP shards and pipeline stages restore onto the same mesh
and can be reassembled offline.  safetensors executes nothing on load.

``restore`` refuses a checkpoint written for a different layout: world size,
every view's offset and shape, and (FSDP) every leaf's sharding names and
global shape must match.  Trainers keep derived device state (fused-engine
bf16 copies, captured hipGraphs); every trainer bound to the state is
invalidated after a restore, so the next step rebuilds it from the restored
masters instead of training on the old weights.
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch
from safetensors.torch import load_file, save_file

from ..runtime import dist as D


def _manifest(state) -> dict:
    P = state.params
    man = {"step": int(state.step), "rng": int(state.rng), "numel": P.numel, "world_size": D.world_size(),
           "rank": D.rank(),
           "views": {n: {"offset": o, "shape": list(s)} for n, (o, s) in P.offsets.items()}}
    sp = state.extra.get("sharded") if hasattr(state, "extra") else None
    if sp is not None:
        for n, pt in sp.part.items():
            man["views"][n].update({"global_shape": list(pt.global_shape), "names": list(pt.names)})
    return man


def save(state, path: str, metrics: Optional[torch.Tensor] = None) -> str:
    os.makedirs(path, exist_ok=True)
    r = D.rank()
    P = state.params
    tensors = {"master": P.master.detach().cpu().contiguous()}
    for k, v in state.opt_state.items():
        tensors[f"opt/{k}"] = v.detach().cpu().contiguous()
    if metrics is not None:
        tensors["metrics"] = metrics.detach().cpu().contiguous()
    f = os.path.join(path, f"rank{r}.safetensors")
    save_file(tensors, f)
    with open(os.path.join(path, f"rank{r}.json"), "w") as fh:
        json.dump(_manifest(state), fh)
    return f


def restore(state, path: str, metrics: Optional[torch.Tensor] = None):
    r = D.rank()
    t = load_file(os.path.join(path, f"rank{r}.safetensors"))
    with open(os.path.join(path, f"rank{r}.json")) as fh:
        man = json.load(fh)
    P = state.params
    _check_layout(man, _manifest(state), path)
    if tuple(t["master"].shape) != tuple(P.master.shape):
        raise ValueError(f"{path}: master buffer {tuple(t['master'].shape)} != {tuple(P.master.shape)}")
    # optimizer state checked BEFORE anything is copied (a mismatch must not leave a
    # half-restored state): same slots (AdamW: count, m, v, ticket; SGD: count, ticket)
    saved_opt = {k[4:]: tuple(v.shape) for k, v in t.items() if k.startswith("opt/")}
    cur_opt = {k: tuple(v.shape) for k, v in state.opt_state.items()}
    if saved_opt != cur_opt:
        raise ValueError(f"{path}: optimizer state {sorted(saved_opt.items())} does not match the live optimizer's "
                         f"{sorted(cur_opt.items())} (different optimizer or layout)")
    P.master.copy_(t["master"].to(P.master.device))
    for k, v in state.opt_state.items():
        v.copy_(t[f"opt/{k}"].to(v.device))
    if metrics is not None and "metrics" in t:
        metrics.copy_(t["metrics"].to(metrics.device))
    P.sync_shadow()
    state.step = man["step"]
    state.rng = man["rng"]
    for tr in bound_trainers(state):
        tr.invalidate()
    return state


def _check_layout(saved: dict, cur: dict, path: str):
    """Same world size, same named views (offset, local shape), same sharding."""
    ws = saved.get("world_size")
    if ws is not None and ws != cur["world_size"]:
        raise ValueError(f"{path}: written by a {ws}-rank job, restoring into {cur['world_size']} ranks")
    if saved["numel"] != cur["numel"]:
        raise ValueError(f"{path}: flat size {saved['numel']} != {cur['numel']} (different model or mesh)")
    sv, cv = saved["views"], cur["views"]
    if set(sv) != set(cv):
        raise ValueError(f"{path}: parameter names differ: {sorted(set(sv) ^ set(cv))}")
    for n, v in cv.items():
        for key in ("offset", "shape", "global_shape", "names"):
            if key in v or key in sv[n]:
                if sv[n].get(key) != v.get(key):
                    raise ValueError(f"{path}: {n} {key} {sv[n].get(key)} != {v.get(key)}")


def bind_trainer(state, trainer):
    """Register ``trainer`` as holding derived state of ``state`` (see ``restore``)."""
    import weakref

    if hasattr(state, "extra"):
        state.extra.setdefault("trainers", []).append(weakref.ref(trainer))


def bound_trainers(state):
    refs = state.extra.get("trainers", []) if hasattr(state, "extra") else []
    return [t for t in (r() for r in refs) if t is not None]
