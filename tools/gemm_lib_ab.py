"""A/B harness: run ``bench.py`` with the model's plain bf16 GEMMs (no epilogue to
fuse) routed to the vendor library (torch.mm -> hipBLASLt) instead of our
``gemm_dma_kernel``.  Measurement only -- the product op ``ops.kernels.gemm`` has
no library dispatch; this wraps it from the outside for the comparison recorded in
profiles/r3_gemm_lib_ab.txt.

    python tools/gemm_lib_ab.py --strategy pp --model transformer --steps 200
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402

_ours = K.gemm
ROUTED = {"lib": 0, "ours": 0}


def _plain(a, b, kw) -> bool:
    keys_default = {"accumulate": False, "alpha": 1.0, "bias": None, "act": "none", "z_out": None, "z_in": None,
                    "act_bwd": "none", "keep_prob": 1.0, "resid": None, "dbias": None, "cfg": -1, "splits": -1,
                    "opt": None, "out_dtype": torch.bfloat16}
    return (a.is_cuda and a.dim() == 2 and not K._GROUP and a.dtype == b.dtype == torch.bfloat16
            and all(kw.get(k, v) == v if not torch.is_tensor(kw.get(k)) else False for k, v in keys_default.items()))


def gemm_lib(a, b, *, a_layout="mk", b_layout="kn", out=None, **kw):
    if _plain(a, b, kw) and (out is None or out.dtype == torch.bfloat16):
        ROUTED["lib"] += 1
        return torch.mm(a if a_layout == "mk" else a.t(), b if b_layout == "kn" else b.t(), out=out)
    ROUTED["ours"] += 1
    return _ours(a, b, a_layout=a_layout, b_layout=b_layout, out=out, **kw)


if __name__ == "__main__":
    K.gemm = gemm_lib
    import bench

    sys.argv = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")] + sys.argv[1:]
    try:
        bench.main()
    finally:
        print(f"[gemm_lib_ab] plain GEMM calls on hipBLASLt: {ROUTED['lib']}, on ours: {ROUTED['ours']}",
              file=sys.stderr)
