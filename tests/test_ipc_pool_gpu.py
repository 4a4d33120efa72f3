"""The pool of IPC-exported buffers (comm/csrc/ipc_pool.hip): a torn-down comm context
returns its exported buffers to the pool, the next context of the same size takes the
same buffers back (zeroed by its create), and no exported page goes back to the driver
during the process's life.  One process; contexts are created without peers (the
exported handles are never opened)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HIP_D2H = 2


def _create(L, cap):
    ctx = ctypes.c_void_p()
    h = (ctypes.c_char * (3 * 64))()
    assert L.jdt_xgmi_create(0, 2, cap, ctypes.byref(ctx), h) == 0
    return ctx


def _read(ptr, n):
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(n, dtype=np.float32)
    assert hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), ctypes.c_size_t(4 * n),
                         HIP_D2H) == 0
    return out


def test_contexts_reuse_pooled_buffers():
    from jax_distributed_tuts_amd.comm import xgmi as X
    from jax_distributed_tuts_amd.ops import _lib

    torch.cuda.set_device(0)
    L = _lib.lib()
    s0 = X.ipc_pool_stats()
    ctx = _create(L, 123_457)
    s1 = X.ipc_pool_stats()
    assert s1["in_use"] == s0["in_use"] + 3 and s1["buffers"] <= s0["buffers"] + 3
    base = L.jdt_xgmi_stage_base(ctx)
    # dirty the staging half 0, tear down, re-create: the same buffer comes back, zeroed
    src = torch.full((1000,), 7.0, device="cuda")
    assert L.jdt_xgmi_stage_write(ctx, 0, ctypes.c_void_p(src.data_ptr()), 1000, None) == 0
    torch.cuda.synchronize()
    assert float(_read(base, 1000).min()) == 7.0
    L.jdt_xgmi_destroy(ctx)
    s2 = X.ipc_pool_stats()
    assert s2["in_use"] == s0["in_use"] and s2["buffers"] == s1["buffers"]
    ctx2 = _create(L, 123_457)
    assert L.jdt_xgmi_stage_base(ctx2) == base and X.ipc_pool_stats()["buffers"] == s1["buffers"]
    assert not _read(base, 1000).any()
    # a different size takes new buffers; both sizes stay pooled
    ctx3 = _create(L, 65_537)
    assert X.ipc_pool_stats()["buffers"] == s1["buffers"] + 3
    L.jdt_xgmi_destroy(ctx3)
    L.jdt_xgmi_destroy(ctx2)
    assert X.ipc_pool_stats()["in_use"] == s0["in_use"]


@pytest.mark.parametrize("ws", [2, 4])
def test_two_phase_teardown_without_pool(tmp_path, ws):
    """Contexts churned with the pool OFF (exported pages back to the driver at every
    teardown) and torch tensors allocated in between: with the two-phase teardown (every
    rank unmaps its peers' pages, a barrier, then every rank frees its own) no self-test
    fails and no canary tensor is written -- the round-5 failure mode (4 ranks, one-call
    teardown) was a rank's own fresh tensors changing under it."""
    from jax_distributed_tuts_amd.runtime.launch import spawn

    from . import xgmi_workers as XW
    from .test_xgmi_gpu import _load

    spawn(XW.ipc_churn, ws, str(tmp_path), gpu=True)
    for r, o in enumerate(_load(tmp_path, "churn", ws)):
        assert o["fails"] == 0 and o["bad"] == 0, (r, o)
        assert o["pool_in_use"] == 0 and o["pool_buffers"] == 0, (r, o)   # nothing kept with the pool off
