"""Checkpoint / resume (the reference has none).

Rank-local files: each rank writes ``<dir>/rank<r>.safetensors`` with its flat
fp32 master, AdamW moments, device step counter and running metrics, plus a
JSON manifest of the named views (name -> offset, local shape, global shape,
sharding names) so FSDP shards and pipeline stages restore onto the same mesh
and can be reassembled offline.  safetensors executes nothing on load.
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
    man = {"step": int(state.step), "rng": int(state.rng), "numel": P.numel,
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
    if man["numel"] != P.numel:
        raise ValueError("checkpoint layout does not match the model/mesh")
    P.master.copy_(t["master"].to(P.master.device))
    for k, v in state.opt_state.items():
        v.copy_(t[f"opt/{k}"].to(v.device))
    if metrics is not None and "metrics" in t:
        metrics.copy_(t["metrics"].to(metrics.device))
    P.sync_shadow()
    state.step = man["step"]
    state.rng = man["rng"]
    return state
