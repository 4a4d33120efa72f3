"""Metrics helpers: (sum, count) metrics and the reference's printer (util.py:170-181).

Metrics are ``{name: (sum, count)}``.  On device the framework keeps them as a
fp32[4] buffer ``[loss_sum, loss_count, correct_sum, acc_count]`` that rides in
the gradient all-reduce bucket; :func:`as_metrics` converts it.
"""
from __future__ import annotations

import textwrap
from typing import Dict, Tuple, Union

import torch

Metrics = Dict[str, Tuple[Union[torch.Tensor, float], ...]]


def print_exception(e: BaseException):
    """util.py:12-14: ``ExcType: msg`` with the type in red (ANSI, no termcolor dep)."""
    name = f"\x1b[31m{type(e).__name__}\x1b[0m"
    print(textwrap.fill(f"{name}: {str(e)}"))


def as_metrics(buf: torch.Tensor) -> Metrics:
    b = buf.detach().float().cpu()
    return {"loss": (b[0], b[1]), "accuracy": (b[2], b[3])}


def format_metrics(metrics: Union[Metrics, torch.Tensor], title: str) -> str:
    if isinstance(metrics, torch.Tensor):
        metrics = as_metrics(metrics)
    lines = []
    for k, v in metrics.items():
        s, c = (float(x) for x in v[:2])
        lines.append(f"{k}: {s / c:.6f}")
    if title:
        title = f" {title} "
        max_len = max(len(title), max(map(len, lines)))
        lines = [title.center(max_len, "=")] + lines
    return "\n".join(lines)


def print_metrics(metrics: Union[Metrics, torch.Tensor], title: str) -> None:
    """Same output format as util.py:170-181 (``k: sum/count`` to 6 decimals under a
    centred ``=`` banner).  The only device->host copy of a run."""
    print(format_metrics(metrics, title))
