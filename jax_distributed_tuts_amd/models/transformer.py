"""Decoder-only transformer LM for the hybrid DP x PP tutorial (BASELINE config #5:
"4-layer transformer hybrid DP=2 x PP=4").  The reference has no transformer;
sizes are ours (documented in README): vocab 2048, d_model 512, 8 heads of 64,
d_ff 2048, seq 128, pre-LN, learned positions, GELU(tanh), untied LM head.

Like models/mlp.py the backward is explicit: every matmul is the gfx950 MFMA
GEMM with fused epilogues (bias, GELU + pre-activation save, residual add on
the forward; GELU' + bias-grad on the backward; fp32 beta=1 weight-grad
accumulation), LayerNorm fwd/bwd kernels fuse the residual-gradient add, and
attention is S = a.QK^T (GEMM reading q/k heads in place from the fused QKV
activation) -> causal softmax kernel -> P.V (GEMM writing heads in place).

A model instance can be a pipeline stage: ``layers`` selects a contiguous
block range, ``has_embed``/``has_head`` mark the first/last stage.
"""
from __future__ import annotations

import contextlib
import os

from dataclasses import dataclass, field
from typing import List, Optional

import torch

from ..ops import kernels as K
from ..utils.flat import FlatParams, ParamSpec

# JDT_EMBED_LN=0: the embedding runs as its own launch (embed_fwd) before the first LN1
_EMBED_LN = os.environ.get("JDT_EMBED_LN", "1") != "0"


@dataclass
class TransformerConfig:
    vocab_size: int = 2048
    d_model: int = 512
    n_heads: int = 8
    d_ff: int = 2048
    seq_len: int = 128
    n_layers: int = 4
    dropout_rate: float = 0.0
    ln_eps: float = 1e-6


@dataclass
class _BlockCache:
    x: torch.Tensor
    h1: torch.Tensor
    m1: torch.Tensor
    r1: torch.Tensor
    qkv: torch.Tensor
    o: torch.Tensor
    P: torch.Tensor
    x2: torch.Tensor
    h2: torch.Tensor
    m2: torch.Tensor
    r2: torch.Tensor
    z1: torch.Tensor
    u: torch.Tensor
    off: int


class WGradArena:
    """Deferred weight gradients (the "W pass" of zero-bubble pipeline schedules): the
    weight-gradient GEMMs of a per-microbatch schedule run ONCE per step over all the
    stage's tokens instead of once per microbatch.  Every microbatch's forward writes
    the GEMM inputs (h1 = LN1(x), o, h2 = LN2(x2), u = GELU(z1), hf = LN_f(x)) and its
    backward the output gradients (dqkv, dx2, dz1, dx3 = d(block output), dlogits) into
    its own rows [i * mb, (i + 1) * mb) of per-layer [T, width] buffers; ``weight_grads``
    then runs dW = A^T . dZ with K = T (the layer-major shapes: 4x the K of a
    microbatch, a quarter of the launches).  The backward chain of a microbatch (the
    pipeline's critical path, dX GEMMs / LayerNorm / attention) no longer waits on them."""

    def __init__(self, model: "TransformerLM", nseq: int, device):
        c = model.cfg
        T, d = nseq * c.seq_len, c.d_model
        self.T, self.nseq = T, nseq
        mk = lambda w: torch.empty(T, w, dtype=torch.bfloat16, device=device)  # noqa: E731
        self.blocks = {l: {"h1": mk(d), "dqkv": mk(3 * d), "o": mk(d), "dx2": mk(d), "h2": mk(d), "dz1": mk(c.d_ff),
                           "u": mk(c.d_ff), "dx3": mk(d)} for l in model.layers}
        self.head = {"hf": mk(d), "dlog": mk(c.vocab_size)} if model.has_head else None

    def rows(self, t: torch.Tensor, i: int, n_mb: int) -> torch.Tensor:
        mb = self.T // n_mb
        return t[i * mb:(i + 1) * mb]


@dataclass
class _Cache:
    inp: torch.Tensor
    nseq: int
    blocks: List[_BlockCache] = field(default_factory=list)
    xf: Optional[torch.Tensor] = None
    hf: Optional[torch.Tensor] = None
    mf: Optional[torch.Tensor] = None
    rf: Optional[torch.Tensor] = None
    seed: int = 0
    keep: float = 1.0
    step: Optional[torch.Tensor] = None
    arena: Optional[WGradArena] = None   # deferred weight gradients: this microbatch's rows
    mb: int = 0
    n_mb: int = 1


class TransformerLM:
    def __init__(self, cfg: TransformerConfig = TransformerConfig(), layers: Optional[range] = None,
                 has_embed: bool = True, has_head: bool = True):
        self.cfg = cfg
        self.layers = range(cfg.n_layers) if layers is None else layers
        self.has_embed, self.has_head = has_embed, has_head
        self.names = [f"block_{l}" for l in self.layers] + (["head"] if has_head else [])

    # ------------------------------------------------------------------ metadata
    @property
    def head_bias_name(self) -> Optional[str]:
        return "head/bias" if self.has_head else None

    def gemm_weight_names(self) -> List[str]:
        """Weights whose gradient is one weight-gradient GEMM per backward pass (the
        candidates for the in-epilogue optimizer, ops.kernels.EpilogueAdamW)."""
        out = []
        for l in self.layers:
            b = f"block_{l}"
            out += [f"{b}/attn/qkv/kernel", f"{b}/attn/out/kernel", f"{b}/mlp/fc1/kernel", f"{b}/mlp/fc2/kernel"]
        return out + (["head/kernel"] if self.has_head else [])

    def input_shape(self, nseq: int):
        return (nseq, self.cfg.seq_len) if self.has_embed else (nseq * self.cfg.seq_len, self.cfg.d_model)

    def input_dtype(self):
        return torch.int32 if self.has_embed else torch.bfloat16

    def output_shape(self, nseq: int):
        c = self.cfg
        return (nseq * c.seq_len, c.vocab_size if self.has_head else c.d_model)

    @staticmethod
    def flatten_labels(y: torch.Tensor) -> torch.Tensor:
        return y.reshape(-1)

    def param_specs(self) -> List[ParamSpec]:
        c = self.cfg
        d = c.d_model
        out = []
        if self.has_embed:
            out += [ParamSpec("embed/wte", (c.vocab_size, d), "normal:0.02"),
                    ParamSpec("embed/wpe", (c.seq_len, d), "normal:0.02")]
        for l in self.layers:
            b = f"block_{l}"
            out += [ParamSpec(f"{b}/ln1/scale", (d,), "ones"), ParamSpec(f"{b}/ln1/bias", (d,), "zeros"),
                    ParamSpec(f"{b}/attn/qkv/kernel", (d, 3 * d)), ParamSpec(f"{b}/attn/qkv/bias", (3 * d,), "zeros"),
                    ParamSpec(f"{b}/attn/out/kernel", (d, d)), ParamSpec(f"{b}/attn/out/bias", (d,), "zeros"),
                    ParamSpec(f"{b}/ln2/scale", (d,), "ones"), ParamSpec(f"{b}/ln2/bias", (d,), "zeros"),
                    ParamSpec(f"{b}/mlp/fc1/kernel", (d, c.d_ff)), ParamSpec(f"{b}/mlp/fc1/bias", (c.d_ff,), "zeros"),
                    ParamSpec(f"{b}/mlp/fc2/kernel", (c.d_ff, d)), ParamSpec(f"{b}/mlp/fc2/bias", (d,), "zeros")]
        if self.has_head:
            out += [ParamSpec("ln_f/scale", (d,), "ones"), ParamSpec("ln_f/bias", (d,), "zeros"),
                    ParamSpec("head/kernel", (d, c.vocab_size)), ParamSpec("head/bias", (c.vocab_size,), "zeros")]
        return out

    # ------------------------------------------------------------------ forward
    def forward(self, P: FlatParams, x: torch.Tensor, *, train: bool = False, seed: int = 0, offset: int = 0,
                step: Optional[torch.Tensor] = None, arena: Optional[WGradArena] = None, mb: int = 0,
                n_mb: int = 1):
        """``arena`` (WGradArena): microbatch ``mb`` of ``n_mb``; the weight-gradient
        GEMMs' inputs go to its rows, ``backward`` then skips the weight gradients and
        ``weight_grads`` runs them once for all microbatches."""
        c = self.cfg
        keep = 1.0 - c.dropout_rate if train else 1.0
        A = (lambda l, k: arena.rows(arena.blocks[l][k], mb, n_mb)) if arena is not None else (lambda l, k: None)  # noqa: E731
        emb = None
        if self.has_embed:
            nseq = x.shape[0]
            tok = x.reshape(-1).contiguous()
            if self.layers and _EMBED_LN:
                # the embedding is built by the first block's LN1 launch (ln_gemm(embed=))
                emb = (tok, P.s("embed/wte"), P.s("embed/wpe"), c.seq_len)
                h = torch.empty(tok.shape[0], c.d_model, dtype=torch.bfloat16, device=tok.device)
            else:
                h = K.embed_fwd(tok, P.s("embed/wte"), P.s("embed/wpe"), c.seq_len)
            cache = _Cache(inp=tok, nseq=nseq, seed=seed, keep=keep, step=step, arena=arena, mb=mb, n_mb=n_mb)
        else:
            nseq = x.shape[0] // c.seq_len
            h = x
            cache = _Cache(inp=x, nseq=nseq, seed=seed, keep=keep, step=step, arena=arena, mb=mb, n_mb=n_mb)
        for l in self.layers:
            b = f"block_{l}"
            # LN1 fused into the QKV projection's A operand (one launch; h1 / stats kept for backward)
            qkv, h1, m1, r1 = K.ln_gemm(h, P.p(f"{b}/ln1/scale"), P.p(f"{b}/ln1/bias"), P.s(f"{b}/attn/qkv/kernel"),
                                        eps=c.ln_eps, bias=P.s(f"{b}/attn/qkv/bias"), y_out=A(l, "h1"), embed=emb)
            emb = None
            o, Pm = K.attention_fwd(qkv, nseq, c.seq_len, c.n_heads, causal=True, o_out=A(l, "o"))
            x2 = K.gemm(o, P.s(f"{b}/attn/out/kernel"), bias=P.s(f"{b}/attn/out/bias"), resid=h)
            z1 = torch.empty(x2.shape[0], c.d_ff, dtype=torch.bfloat16, device=x2.device)
            off = int(offset) + (l << 1)
            # LN2 fused into fc1 (bias + GELU epilogue, pre-activation z1 saved)
            u, h2, m2, r2 = K.ln_gemm(x2, P.p(f"{b}/ln2/scale"), P.p(f"{b}/ln2/bias"), P.s(f"{b}/mlp/fc1/kernel"),
                                      eps=c.ln_eps, bias=P.s(f"{b}/mlp/fc1/bias"), act="gelu", z_out=z1,
                                      keep_prob=keep, seed=seed, offset=off, step=step, y_out=A(l, "h2"),
                                      out=A(l, "u"))
            x3 = K.gemm(u, P.s(f"{b}/mlp/fc2/kernel"), bias=P.s(f"{b}/mlp/fc2/bias"), resid=x2)
            cache.blocks.append(_BlockCache(h, h1, m1, r1, qkv, o, Pm, x2, h2, m2, r2, z1, u, off))
            h = x3
        if self.has_head:
            logits, hf, mf, rf = K.ln_gemm(h, P.p("ln_f/scale"), P.p("ln_f/bias"), P.s("head/kernel"),
                                           eps=c.ln_eps, bias=P.s("head/bias"),
                                           y_out=arena.rows(arena.head["hf"], mb, n_mb) if arena is not None else None)
            cache.xf, cache.hf, cache.mf, cache.rf = h, hf, mf, rf
            h = logits
        return h, cache

    # ------------------------------------------------------------------ backward
    def backward(self, P: FlatParams, cache: _Cache, dout: torch.Tensor, *, dout_is_dz: bool = True,
                 need_dx: bool = False, on_ready=None, wgrad=None, opt=None, after=None) -> Optional[torch.Tensor]:
        """``wgrad`` (ops.kernels.WGradStream): run the weight-gradient GEMMs on its
        side stream; the caller joins it before reading the grads.  ``opt``
        (ops.kernels.EpilogueAdamW): this pass carries the weights' final gradients of
        the step -- AdamW runs in the epilogues of their weight-gradient GEMMs.
        A cache with a WGradArena (deferred weight gradients): only the input-gradient
        chain runs here, the GEMM output gradients go to the arena and the caller runs
        ``weight_grads`` once after the last microbatch."""
        if on_ready is not None:
            wgrad = None  # bucket callbacks fire as soon as a layer's grads are queued
        c = self.cfg
        ar = cache.arena
        if ar is not None:
            assert opt is None and on_ready is None, "deferred weight gradients: optimizer runs in weight_grads"
        R = (lambda l, k: ar.rows(ar.blocks[l][k], cache.mb, cache.n_mb)) if ar is not None else (lambda l, k: None)  # noqa: E731
        ready = on_ready if on_ready is not None else (lambda names: None)
        after = after if after is not None else (lambda part: None)   # part's deferred dW inputs complete
        layers = list(self.layers)

        def dw_dx(name, dw, dx):
            if ar is not None:
                return dx()   # the weight gradient is deferred to weight_grads
            return _dw_dx(opt, name, dw, dx)

        fc2_bias = lambda l: P.g(f"block_{l}/mlp/fc2/bias")  # noqa: E731
        if self.has_head:
            if ar is not None:
                _into(ar.rows(ar.head["dlog"], cache.mb, cache.n_mb), dout)
            # dlogits (CE already added the head bias grad); the LN-bwd also reduces
            # the top block's fc2 bias grad (colsum of the residual gradient)
            dhf = dw_dx("head/kernel",
                        lambda: K.dw_gemm(wgrad, cache.hf, dout, P.g("head/kernel"), opt=opt, name="head/kernel"),
                        lambda: K.gemm(dout, P.s("head/kernel"), b_layout="nk"))
            after("head")   # after the dX GEMM: an epilogue AdamW rewrites the shadow it reads
            dx = K.layernorm_bwd(dhf, cache.xf, cache.mf, cache.rf, P.p("ln_f/scale"), P.g("ln_f/scale"),
                                 P.g("ln_f/bias"), dsum=fc2_bias(layers[-1]) if layers else None,
                                 dx_out=R(layers[-1], "dx3") if layers else None)
            fc2_done = True
            ready(["head/kernel", "head/bias", "ln_f/scale", "ln_f/bias"])
        else:
            dx = dout
            if ar is not None and layers:
                dx = _into(R(layers[-1], "dx3"), dout)
            fc2_done = False  # stage boundary: dx arrived from the next stage
        for idx in range(len(layers) - 1, -1, -1):
            l, bc = layers[idx], cache.blocks[idx]
            b = f"block_{l}"
            # x3 = x2 + u.W2 + b2
            if not fc2_done:
                K.colsum_(dx, P.g(f"{b}/mlp/fc2/bias"))
            n2, n1 = f"{b}/mlp/fc2/kernel", f"{b}/mlp/fc1/kernel"
            dz1 = dw_dx(n2, lambda: K.dw_gemm(wgrad, bc.u, dx, P.g(n2), opt=opt, name=n2),
                        lambda: K.gemm(dx, P.s(n2), b_layout="nk", z_in=bc.z1, act_bwd="gelu",
                                       keep_prob=cache.keep, seed=cache.seed, offset=bc.off, step=cache.step,
                                       dbias=P.g(f"{b}/mlp/fc1/bias"), out=R(l, "dz1")))
            dh2 = dw_dx(n1, lambda: K.dw_gemm(wgrad, bc.h2, dz1, P.g(n1), opt=opt, name=n1),
                        lambda: K.gemm(dz1, P.s(n1), b_layout="nk"))
            # x2 = x + o.Wo + bo: the LN2-bwd output dx2 is also Wo's bias grad
            dx2 = K.layernorm_bwd(dh2, bc.x2, bc.m2, bc.r2, P.p(f"{b}/ln2/scale"), P.g(f"{b}/ln2/scale"),
                                  P.g(f"{b}/ln2/bias"), dres=dx, dsum=P.g(f"{b}/attn/out/bias"), dx_out=R(l, "dx2"))
            no, nq = f"{b}/attn/out/kernel", f"{b}/attn/qkv/kernel"
            do = dw_dx(no, lambda: K.dw_gemm(wgrad, bc.o, dx2, P.g(no), opt=opt, name=no),
                       lambda: K.gemm(dx2, P.s(no), b_layout="nk"))
            dqkv = K.attention_bwd(do, bc.qkv, bc.P, cache.nseq, c.seq_len, c.n_heads, o=bc.o,
                                   dbias=P.g(f"{b}/attn/qkv/bias"), dqkv=R(l, "dqkv"))
            dh1 = dw_dx(nq, lambda: K.dw_gemm(wgrad, bc.h1, dqkv, P.g(nq), opt=opt, name=nq),
                        lambda: K.gemm(dqkv, P.s(nq), b_layout="nk"))
            below = fc2_bias(layers[idx - 1]) if idx > 0 else None  # next (lower) block's fc2 bias grad
            dx = K.layernorm_bwd(dh1, bc.x, bc.m1, bc.r1, P.p(f"{b}/ln1/scale"), P.g(f"{b}/ln1/scale"),
                                 P.g(f"{b}/ln1/bias"), dres=dx2, dsum=below,
                                 dx_out=R(layers[idx - 1], "dx3") if idx > 0 else None)
            fc2_done = below is not None
            after(l)
            ready([s.name for s in self.param_specs() if s.name.startswith(b + "/")])
        if self.has_embed:
            K.embed_bwd(dx, cache.inp, P.g("embed/wte"), P.g("embed/wpe"), c.seq_len)
            ready(["embed/wte", "embed/wpe"])
            return None
        return dx if need_dx else None

    def weight_grads(self, P: FlatParams, arena: WGradArena, *, wgrad=None, opt=None, on=None):
        """The deferred weight gradients of every microbatch in one GEMM per weight:
        dW (+)= A^T . dZ over all T = n_mb * mb rows of ``arena`` (``opt``: AdamW in the
        epilogue, each weight's single gradient contribution of the step).  ``on(j)``:
        context for GEMM j (parallel.pipeline._MbStreams: the GEMMs touch disjoint
        weights and only read the step counter, so they may run on several streams)."""
        if opt is not None:
            opt.only_contribution = True
        order = []
        if self.has_head:
            order.append(("head/kernel", arena.head["hf"], arena.head["dlog"]))
        for l in reversed(list(self.layers)):
            a, b = arena.blocks[l], f"block_{l}"
            order += [(f"{b}/mlp/fc2/kernel", a["u"], a["dx3"]), (f"{b}/mlp/fc1/kernel", a["h2"], a["dz1"]),
                      (f"{b}/attn/out/kernel", a["o"], a["dx2"]), (f"{b}/attn/qkv/kernel", a["h1"], a["dqkv"])]
        for j, (name, h, dz) in enumerate(order):
            with (on(j) if on is not None else contextlib.nullcontext()):
                K.dw_gemm(wgrad, h, dz, P.g(name), opt=opt, name=name)

    def weight_grads_of(self, P: FlatParams, arena: WGradArena, part, *, opt=None, on=None, j0: int = 0) -> int:
        """The deferred weight-gradient GEMMs of one ``part`` ("head" or a layer index),
        as soon as the backward chain has produced that part's output gradients (the
        ``after`` hook of ``backward``); GEMM j runs under ``on(j0 + j)``.  Returns the
        next j0."""
        if opt is not None:
            opt.only_contribution = True
        order = self.weight_grad_items(arena, part)
        for j, (name, h, dz) in enumerate(order):
            with (on(j0 + j) if on is not None else contextlib.nullcontext()):
                K.dw_gemm(None, h, dz, P.g(name), opt=opt, name=name)
        return j0 + len(order)

    @staticmethod
    def weight_grad_items(arena: WGradArena, part):
        """(weight name, A rows, dZ rows) of one part's deferred weight-gradient GEMMs,
        in the W pass's order (``weight_grads_of``)."""
        if part == "head":
            return [("head/kernel", arena.head["hf"], arena.head["dlog"])]
        a, b = arena.blocks[part], f"block_{part}"
        return [(f"{b}/mlp/fc2/kernel", a["u"], a["dx3"]), (f"{b}/mlp/fc1/kernel", a["h2"], a["dz1"]),
                (f"{b}/attn/out/kernel", a["o"], a["dx2"]), (f"{b}/attn/qkv/kernel", a["h1"], a["dqkv"])]

    def sync_groups(self):
        """The stage's parameters cut into groups that become final one at a time in the
        W pass: (key, first parameter) in W-pass order -- "embed" (its gradient is final
        when the backward chain ends), then one group per weight-gradient GEMM, keyed by
        the weight: the GEMM's weight plus the bias / LayerNorm parameters that follow it
        in the flat layout up to the next group (computed by the chain, already final);
        a layer's qkv group starts at its ln1 (parallel/pipeline.py _sync_buckets)."""
        out = [("embed", "embed/wte")] if self.has_embed else []
        if self.has_head:
            out.append(("head/kernel", "ln_f/scale"))
        for l in reversed(list(self.layers)):
            b = f"block_{l}"
            out += [(f"{b}/mlp/fc2/kernel", f"{b}/mlp/fc2/kernel"), (f"{b}/mlp/fc1/kernel", f"{b}/mlp/fc1/kernel"),
                    (f"{b}/attn/out/kernel", f"{b}/attn/out/kernel"), (f"{b}/attn/qkv/kernel", f"{b}/ln1/scale")]
        return out


def _into(dst: Optional[torch.Tensor], src: torch.Tensor) -> torch.Tensor:
    """``src`` placed in ``dst`` (no copy when it already is ``dst``)."""
    if dst is None:
        return src
    if dst.data_ptr() != src.data_ptr():
        dst.copy_(src)
    return dst


def _dw_dx(opt, name: str, dw, dx):
    """A Dense layer's weight gradient ``dw()`` and input gradient ``dx()`` (both only
    need dz): one grouped launch.  With the in-epilogue optimizer covering the weight
    (ops.kernels.EpilogueAdamW), the input gradient runs FIRST and alone -- it reads the
    weight's bf16 shadow, which the weight-gradient GEMM's epilogue then overwrites."""
    if opt is not None and opt.covers(name):
        out = dx()
        dw()
        return out
    with K.gemm_group():
        dw()
        return dx()


def lm_stage(cfg: TransformerConfig, n_stages: int, stage: int) -> TransformerLM:
    from ..parallel.pipeline import split_layers

    r = split_layers(cfg.n_layers, n_stages)[stage]
    return TransformerLM(cfg, layers=r, has_embed=stage == 0, has_head=stage == n_stages - 1)
