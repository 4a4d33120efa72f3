"""ctypes binding to the in-tree gfx950 kernel library.

The library is loaded lazily on the first GPU op.  On a machine with a GPU the
HIP path is mandatory: if the library is missing or fails to load, the op
raises instead of silently falling back to eager PyTorch (CPU tensors use the
pure-torch reference implementations in ``ops/kernels.py``; those exist for the
gloo simulation mode and as the numerics oracle in tests).
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import c_float, c_int, c_long, c_ulonglong, c_void_p

from . import build as _build

_lock = threading.Lock()
_lib = None


class GemmArgs(ctypes.Structure):
    """Mirror of ``jdt::GemmArgs`` in csrc/gemm.hip (field order and types must match)."""

    _fields_ = [
        ("A", c_void_p), ("lda", c_long), ("sA", c_long), ("a_f32", c_int), ("a_trans", c_int),
        ("B", c_void_p), ("ldb", c_long), ("sB", c_long), ("b_f32", c_int), ("b_trans", c_int),
        ("M", c_int), ("N", c_int), ("K", c_int), ("alpha", c_float),
        ("bias", c_void_p), ("bias_f32", c_int), ("act", c_int),
        ("Zout", c_void_p), ("ldz", c_long), ("sZ", c_long),
        ("Zin", c_void_p), ("ldzin", c_long), ("sZin", c_long), ("act_bwd", c_int),
        ("keep_prob", c_float), ("seed", c_ulonglong), ("offset", c_ulonglong),
        ("resid", c_void_p), ("ldr", c_long), ("sR", c_long),
        ("dbias", c_void_p),
        ("C", c_void_p), ("ldc", c_long), ("sC", c_long), ("c_f32", c_int), ("accumulate", c_int),
        ("step_ptr", c_void_p),
        ("zin", c_int), ("sA2", c_long), ("sB2", c_long), ("sC2", c_long),
        ("opt_p", c_void_p), ("opt_m", c_void_p), ("opt_v", c_void_p), ("opt_s", c_void_p), ("opt_step", c_void_p),
        ("opt_lr", c_float), ("opt_b1", c_float), ("opt_b2", c_float), ("opt_eps", c_float), ("opt_wd", c_float),
        ("opt_gs", c_float),
        ("seed_ptr", c_void_p),
    ]


class LnArgs(ctypes.Structure):
    """Mirror of ``jdt::LnArgs`` in csrc/gemm.hip (LayerNorm fused into a GEMM's A operand)."""

    _fields_ = [("X", c_void_p), ("ldx", c_long), ("gamma", c_void_p), ("beta", c_void_p), ("eps", c_float),
                ("Y", c_void_p), ("ldy", c_long), ("mean", c_void_p), ("rstd", c_void_p)]


_SIGS = {
    "jdt_gemm_ln": (c_int, [ctypes.POINTER(GemmArgs), ctypes.POINTER(LnArgs), c_void_p]),
    "jdt_gemm_ln_eligible": (c_int, [ctypes.POINTER(GemmArgs), ctypes.POINTER(LnArgs)]),
    "jdt_ln_args_size": (c_int, []),
    "jdt_gemm_ln_set_cfg": (None, [c_int]),
    "jdt_adamw_ranges": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_long,
                                 c_float, c_float, c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    "jdt_gemm": (c_int, [ctypes.POINTER(GemmArgs), c_int, c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p]),
    "jdt_gemm_args_size": (c_int, []),
    "jdt_gemm_set_wt": (c_int, [c_int]),
    "jdt_gemm_group": (c_int, [ctypes.POINTER(GemmArgs), c_int, c_void_p, c_long, c_void_p, c_long, c_void_p]),
    "jdt_gemm_wpass_table_bytes": (c_int, []),
    "jdt_gemm_wpass_plan": (c_int, [ctypes.POINTER(GemmArgs), c_int, c_int, c_void_p, c_void_p, c_long, c_void_p,
                                    c_long]),
    "jdt_gemm_wpass_launch": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "jdt_gemm_set_group_split": (None, [c_int]),
    "jdt_gemm_set_group_tile": (None, [c_int]),
    "jdt_ln_set_rows": (None, [c_int]),
    "jdt_ln_set_waves": (None, [c_int]),
    "jdt_ln_set_xcd": (None, [c_int]),
    "jdt_attn128_set_xcd": (None, [c_int]),
    "jdt_attn128_set_stamps": (None, [c_void_p]),
    "jdt_gemm_set_group_m": (None, [c_int]),
    "jdt_gemm_set_epi_vec": (None, [c_int]),
    "jdt_gemm_set_epi_vec_min": (None, [c_long]),
    "jdt_gemm_set_r": (None, [c_int]),
    "jdt_gemm_set_tune": (None, [c_int]),
    "jdt_flash_set_head": (None, [c_int]),
    "jdt_flash_set_attn128": (None, [c_int]),
    "jdt_xent_set_rpw": (None, [c_int]),
    "jdt_gemm_set_preload": (None, [c_int]),
    "jdt_gemm_set_exact": (None, [c_int]),
    "jdt_gemm_set_dma": (None, [c_int]),
    "jdt_xent": (c_int, [c_void_p, c_int, c_long, c_void_p, c_int, c_int, c_float, c_void_p, c_long, c_void_p,
                         c_void_p, c_void_p, c_void_p]),
    "jdt_adamw": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_float, c_float, c_float,
                          c_float, c_float, c_float, c_void_p, c_void_p, c_int, c_void_p]),
    "jdt_sgd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_float, c_float, c_float, c_float,
                        c_void_p, c_void_p, c_int, c_void_p]),
    "jdt_cast_f32_bf16": (c_int, [c_void_p, c_void_p, c_long, c_void_p]),
    "jdt_scale": (c_int, [c_void_p, c_long, c_float, c_void_p]),
    "jdt_act_bwd": (c_int, [c_void_p, c_void_p, c_int, c_float, c_ulonglong, c_ulonglong, c_void_p, c_void_p, c_int, c_int,
                            c_void_p, c_void_p, c_void_p]),
    "jdt_metrics_fold": (c_int, [c_void_p, c_void_p, c_int, c_void_p]),
    "jdt_metrics_fold_slab": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "jdt_xent_slab": (c_int, [c_void_p, c_int, c_long, c_void_p, c_int, c_int, c_float, c_void_p, c_long, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "jdt_ln_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float,
                           c_void_p]),
    "jdt_ln_fwd_embed": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_int, c_int, c_float, c_void_p]),
    "jdt_ln_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_int, c_int, c_void_p]),
    "jdt_attn_softmax_fwd": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "jdt_attn_softmax_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "jdt_embed_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "jdt_embed_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "jdt_colsum": (c_int, [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p]),
    "jdt_flash_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int, c_void_p]),
    "jdt_flash_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                              c_int, c_int, c_float, c_int, c_void_p]),
}


def _declare(lib):
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    # optional symbols declared by other modules register themselves via `declare`
    return lib


_extra_sigs: dict = {}


def declare(name: str, restype, argtypes):
    """Register a signature for a launcher defined in another csrc file."""
    _extra_sigs[name] = (restype, argtypes)
    if _lib is not None:
        fn = getattr(_lib, name)
        fn.restype, fn.argtypes = restype, argtypes


def lib():
    """Load (building first if the .so is missing/stale and a compiler exists)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = _build.LIB
        if (not path.exists()) or (os.environ.get("JDT_AUTOBUILD", "1") == "1" and _build.is_stale()):
            try:
                _build.build(verbose=True)
            except Exception as e:  # noqa: BLE001
                if not path.exists():
                    raise RuntimeError(f"gfx950 kernel library {path} is missing and could not be built: {e}") from e
        l = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        _declare(l)
        for name, (res, args) in _extra_sigs.items():
            fn = getattr(l, name)
            fn.restype, fn.argtypes = res, args
        if l.jdt_gemm_args_size() != ctypes.sizeof(GemmArgs):
            raise RuntimeError("GemmArgs layout mismatch between Python and csrc/gemm.hip")
        if os.environ.get("JDT_GROUP_SPLIT") == "0":   # A/B: no split-K inside grouped GEMM launches
            l.jdt_gemm_set_group_split(0)
        if os.environ.get("JDT_GEMM_TUNE") == "0":  # A/B: heuristic tile choice only
            l.jdt_gemm_set_tune(0)
        if os.environ.get("JDT_GEMM_EPI_VEC") == "0":  # A/B: per-element GEMM epilogue
            l.jdt_gemm_set_epi_vec(0)
        if os.environ.get("JDT_GEMM_EPI_MIN"):  # A/B: vectorised epilogue only from this many outputs
            l.jdt_gemm_set_epi_vec_min(int(os.environ["JDT_GEMM_EPI_MIN"]))
        if os.environ.get("JDT_GEMM_R"):  # A/B: force the LDS-DMA GEMM's sub-tiles per ring slot
            l.jdt_gemm_set_r(int(os.environ["JDT_GEMM_R"]))
        if os.environ.get("JDT_GEMM_GROUP_M"):  # A/B: LDS-DMA GEMM tile order in row-groups of G tiles
            l.jdt_gemm_set_group_m(int(os.environ["JDT_GEMM_GROUP_M"]))
        if os.environ.get("JDT_GEMM_WT"):  # A/B: write-through GEMM epilogue stores (1: C / Zout, 2: AdamW, 3: both)
            check(l.jdt_gemm_set_wt(int(os.environ["JDT_GEMM_WT"])), "jdt_gemm_set_wt")
        if os.environ.get("JDT_LN_GEMM_CFG"):  # A/B: force the LN-fused GEMM's tile (any row count; 0 = heuristic)
            l.jdt_gemm_ln_set_cfg(int(os.environ["JDT_LN_GEMM_CFG"]))
        if os.environ.get("JDT_LN_WAVES"):  # A/B: force LayerNorm-backward waves per workgroup (0 = auto)
            l.jdt_ln_set_waves(int(os.environ["JDT_LN_WAVES"]))
        if os.environ.get("JDT_XENT_RPW"):  # A/B: force the wide-vocabulary CE kernel's rows per wave
            l.jdt_xent_set_rpw(int(os.environ["JDT_XENT_RPW"]))
        if os.environ.get("JDT_LN_ROWS"):  # A/B: force LayerNorm-backward rows per wave (0 = auto)
            l.jdt_ln_set_rows(int(os.environ["JDT_LN_ROWS"]))
        if os.environ.get("JDT_LN_XCD"):  # A/B: 0 = LayerNorm row blocks in natural order (not XCD-contiguous)
            l.jdt_ln_set_xcd(int(os.environ["JDT_LN_XCD"]))
        if os.environ.get("JDT_ATTN_XCD"):  # A/B: 0 = attention forward tiles in natural order
            l.jdt_attn128_set_xcd(int(os.environ["JDT_ATTN_XCD"]))
        _lib = l
        return _lib


def check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")


def stream_ptr(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream

