"""Wide-vocabulary softmax-CE (fwd + bwd + metrics, bias-gradient column sums) on
the transformer LM head's shape (2048 tokens x 2048 classes, bf16): rows per wave
sweep, and without the column sums.  Each timing: 50 launches in one hipGraph,
median of 5.

    python tools/bench_xent.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.ops import _lib  # noqa: E402
from jax_distributed_tuts_amd.ops import kernels as K  # noqa: E402
from tools.bench_gemm import timed  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for M, C in ((2048, 2048), (512, 2048)):
        z = torch.randn(M, C, device=dev).to(torch.bfloat16)
        lab = torch.randint(0, C, (M,), device=dev, dtype=torch.int32)
        dl = torch.empty_like(z)
        db = torch.zeros(C, device=dev)
        met = torch.zeros(4, device=dev)
        row = []
        for r in (0, 1, 2, 4, 8):
            _lib.lib().jdt_xent_set_rpw(r)
            t = timed(lambda: K.softmax_xent(z, lab, grad_scale=1.0 / M, dlogits=dl, dbias=db, metrics=met))
            row.append(f"rpw={r or 'auto'}: {t:6.2f}")
        _lib.lib().jdt_xent_set_rpw(0)
        t_nb = timed(lambda: K.softmax_xent(z, lab, grad_scale=1.0 / M, dlogits=dl, metrics=met))
        t_nm = timed(lambda: K.softmax_xent(z, lab, grad_scale=1.0 / M, dlogits=dl))
        rl = torch.empty(M, device=dev)
        t_f = timed(lambda: K.softmax_xent(z, lab, row_loss=rl))
        print(f"xent M={M} C={C}: " + " | ".join(row) + f" | no dbias {t_nb:6.2f} | no dbias/metrics {t_nm:6.2f}"
              f" | loss only {t_f:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
