"""Named scopes for profilers (reference: jax.named_scope at data_paral.py:210,220;
param_sharding.py:58,146,350,355).

``named_scope(name)`` is a context manager / decorator that opens a
``torch.profiler.record_function`` range and a ROCTx range
(``roctxRangePushA/Pop`` from librocprofiler-sdk-roctx / libroctx64), so
``rocprofv3 --marker-trace`` shows the same region names as the reference
(``sync_grads``, ``sync_metrics``, ``shard_params``, ``gather_params``...).
ROCTx is optional: without the library only the torch range is emitted.
Under hipGraph capture the ranges mark capture time, not replay; replays are
bracketed by ``replay_scope("<step program>[graph xS]")`` instead (the scopes
inside a replayed step are the kernels of the trace, in capture order).
"""
from __future__ import annotations

import contextlib
import ctypes
import functools
import os
import time

import torch

_roctx = None
_roctx_tried = False


def _get_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("JDT_ROCTX", "1") != "1":
        return None
    for name in ("librocprofiler-sdk-roctx.so", "libroctx64.so", "/opt/rocm/lib/librocprofiler-sdk-roctx.so",
                 "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            break
        except (OSError, AttributeError):
            continue
    return _roctx


def _torch_profiling() -> bool:
    return bool(torch.autograd.profiler._is_profiler_enabled)


class named_scope(contextlib.ContextDecorator):
    """The torch range is opened only while a torch profiler is recording: entering a
    ``record_function`` costs ~10-25 us of host time, which sat inside every timed
    hipGraph replay (bench.py's 20-step driver form is ~270 us of GPU time); the ROCTx
    range (~1 us) is always emitted."""

    def __init__(self, name: str):
        self.name = name
        self._rf = None

    def __enter__(self):
        if _torch_profiling():
            self._rf = torch.profiler.record_function(self.name)
            self._rf.__enter__()
        r = _get_roctx()
        if r is not None:
            r.roctxRangePushA(self.name.encode())
        return self

    def __exit__(self, *exc):
        r = _get_roctx()
        if r is not None:
            r.roctxRangePop()
        if self._rf is not None:
            self._rf.__exit__(*exc)
            self._rf = None
        return False


def replay_scope(name: str, steps: int = 1) -> "named_scope":
    """Range around a hipGraph replay of ``steps`` captured training steps."""
    return named_scope(f"{name}[graph x{steps}]")


class StepTimer:
    """hipEvent-pair step timer (GPU) / perf_counter (CPU) feeding steps/sec reports."""

    def __init__(self, device):
        self.gpu = torch.device(device).type == "cuda"
        self.times_ms = []

    @contextlib.contextmanager
    def step(self):
        if self.gpu:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            b.synchronize()
            self.times_ms.append(a.elapsed_time(b))
        else:
            t = time.perf_counter()
            yield
            self.times_ms.append((time.perf_counter() - t) * 1e3)

    def percentile(self, q: float) -> float:
        if not self.times_ms:
            return float("nan")
        s = sorted(self.times_ms)
        return s[min(len(s) - 1, int(q / 100.0 * len(s)))]
