"""Autograd wrappers of the gfx950 kernels, for user-written, flax-style code.

The trainers run explicit, hand-scheduled backward passes (models/mlp.py).  A
user porting the reference writes a *differentiable* ``loss_fn(params,
apply_fn, batch, rng)`` instead (reference data_paral.py:171-189, consumed by
``jax.value_and_grad`` at util.py:53,65-67).  ``dense`` makes that possible on
the same kernels: its forward is ONE GEMM launch with the bias / activation /
dropout epilogue (``ops.kernels.gemm``), its backward regenerates the dropout
mask and act' from the saved bf16 pre-activation (``act_bwd``, which also
produces the bias gradient) and runs the dX and dW GEMMs -- HIP kernels on GPU,
the torch reference ops on CPU.  Numerics follow flax ``Dense(dtype=bf16)``:
bf16 operands, fp32 accumulation, bf16 activations, fp32 master weights and
gradients.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import kernels as K


class _Dense(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act: str, keep: float, seed: int, offset: int, seed_dev=None):
        M = x.shape[0]
        out = torch.empty(M, w.shape[1], dtype=torch.bfloat16, device=x.device)
        hid = act != "none" or keep < 1.0
        z = torch.empty_like(out) if hid else None
        # flax Dense(dtype=bf16) casts its input: do it once, the dW GEMM reuses it
        xin = x.detach().contiguous()
        if xin.dtype != torch.bfloat16:
            xin = K.cast_bf16_(xin.float(), torch.empty(xin.shape, dtype=torch.bfloat16, device=xin.device))
        K.gemm(xin, w.detach(), a_layout="mk", b_layout="kn", out=out, bias=b.detach(),
               act=act, z_out=z, keep_prob=keep, seed=seed, offset=offset, seed_dev=seed_dev)
        ctx.save_for_backward(xin, w, z)
        ctx.cfg = (act, keep, seed, offset, x.dtype)
        ctx.seed_dev = seed_dev
        return out

    @staticmethod
    def backward(ctx, dout):
        xin, w, z = ctx.saved_tensors
        act, keep, seed, offset, xdtype = ctx.cfg
        dz = dout.to(torch.bfloat16).contiguous()
        db = torch.zeros(w.shape[1], dtype=torch.float32, device=dz.device)
        # dz = dout * mask/keep * act'(z) and db = colsum(dz) in one pass (any width)
        dz = K.act_bwd(dz, z, act, keep_prob=keep, seed=seed, offset=offset, dbias=db, seed_dev=ctx.seed_dev)
        dx = dw = None
        if ctx.needs_input_grad[1]:
            dw = torch.zeros(w.shape, dtype=torch.float32, device=dz.device)
            K.gemm(xin, dz, a_layout="km", b_layout="kn", out=dw, accumulate=True)
        if ctx.needs_input_grad[0]:
            dx = torch.empty(xin.shape[0], w.shape[0], dtype=torch.bfloat16, device=dz.device)
            K.gemm(dz, w.detach(), a_layout="mk", b_layout="nk", out=dx)
            dx = dx.to(xdtype)
        return dx, dw, db if ctx.needs_input_grad[2] else None, None, None, None, None, None


def dense(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, *, act: str = "none", keep: float = 1.0,
          seed: int = 0, offset: int = 0, seed_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``dropout(act(bf16(x) @ bf16(w) + b))`` as a bf16 [M, N] tensor, differentiable
    w.r.t. x, w (fp32 [in, out]) and b.  Dropout keeps with probability ``keep``
    under Philox stream (seed, offset) -- the same masks the engine draws.
    ``seed_dev``: device int64[1] seed read by the kernels instead of ``seed``."""
    return _Dense.apply(x, w, b, act, float(keep), int(seed) & 0xFFFFFFFFFFFFFFFF, int(offset), seed_dev)


class _SoftmaxXent(torch.autograd.Function):
    """Per-row softmax cross-entropy on the fused xent kernel (csrc/xent.hip): ONE
    launch computes the row losses AND d(row loss)/dlogits = softmax - onehot
    (saved, bf16 like the trainers' dlogits); the backward only scales each row by
    its upstream gradient (1/B for a ``loss.mean()``)."""

    @staticmethod
    def forward(ctx, logits, labels):
        M, C = logits.shape
        lg = logits.detach()
        if lg.stride(-1) != 1:
            lg = lg.contiguous()
        lab = labels.detach().to(torch.int32).contiguous()
        gpu = lg.is_cuda
        d = torch.empty(M, C, dtype=torch.bfloat16 if gpu else torch.float32, device=lg.device)
        loss = torch.empty(M, dtype=torch.float32, device=lg.device)
        K.softmax_xent(lg, lab, grad_scale=1.0, dlogits=d, row_loss=loss)
        ctx.save_for_backward(d)
        ctx.ldtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, gloss):
        (d,) = ctx.saved_tensors
        return (d.float() * gloss.float()[:, None]).to(ctx.ldtype), None


def softmax_cross_entropy_with_integer_labels(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """optax.softmax_cross_entropy_with_integer_labels: per-row CE (fp32), forward and
    gradient from the fused HIP xent kernel (torch reference ops on CPU)."""
    return _SoftmaxXent.apply(logits, labels)
