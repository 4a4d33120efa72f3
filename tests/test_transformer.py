"""Transformer LM: explicit fused backward == torch autograd of the same maths
(CPU reference path, tiny config), and the pipeline split trains the same model."""
import math

import pytest
import torch

from jax_distributed_tuts_amd.models.mlp import loss_and_grad
from jax_distributed_tuts_amd.models.transformer import TransformerConfig, TransformerLM, lm_stage
from jax_distributed_tuts_amd.parallel.pipeline_lm import lm_batch
from jax_distributed_tuts_amd.utils.flat import FlatParams

CFG = TransformerConfig(vocab_size=64, d_model=64, n_heads=4, d_ff=128, seq_len=16, n_layers=2)


def autograd_reference(P: FlatParams, cfg, tok, labels):
    """fp32 functional transformer with torch autograd."""
    ps = {n: P.p(n).detach().clone().requires_grad_() for n in P.names()}
    B, S = tok.shape
    d, H = cfg.d_model, cfg.n_heads
    Dh = d // H

    def ln(x, g, b):
        return torch.nn.functional.layer_norm(x, (d,), g, b, eps=cfg.ln_eps)

    x = ps["embed/wte"][tok.long()] + ps["embed/wpe"][None]
    x = x.reshape(B * S, d)
    for l in range(cfg.n_layers):
        b = f"block_{l}"
        h = ln(x, ps[f"{b}/ln1/scale"], ps[f"{b}/ln1/bias"])
        qkv = h @ ps[f"{b}/attn/qkv/kernel"] + ps[f"{b}/attn/qkv/bias"]
        q, k, v = qkv.view(B, S, 3, H, Dh).permute(2, 0, 3, 1, 4)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(Dh)
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool), 1), float("-inf"))
        o = (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(B * S, d)
        x = x + o @ ps[f"{b}/attn/out/kernel"] + ps[f"{b}/attn/out/bias"]
        h2 = ln(x, ps[f"{b}/ln2/scale"], ps[f"{b}/ln2/bias"])
        u = torch.nn.functional.gelu(h2 @ ps[f"{b}/mlp/fc1/kernel"] + ps[f"{b}/mlp/fc1/bias"], approximate="tanh")
        x = x + u @ ps[f"{b}/mlp/fc2/kernel"] + ps[f"{b}/mlp/fc2/bias"]
    hf = ln(x, ps["ln_f/scale"], ps["ln_f/bias"])
    logits = hf @ ps["head/kernel"] + ps["head/bias"]
    loss = torch.nn.functional.cross_entropy(logits, labels.reshape(-1).long())
    loss.backward()
    return loss.detach(), {n: t.grad for n, t in ps.items()}


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def test_transformer_grads_match_autograd():
    model = TransformerLM(CFG)
    P = FlatParams(model.param_specs()).init_(0)
    batch = lm_batch(CFG, global_batch=2, seed=3)
    m = torch.zeros(4)
    loss_and_grad(model, P, batch.inputs, batch.labels, train=False, seed=0, offset=0, step=None, metrics=m)
    ref_loss, ref_g = autograd_reference(P, CFG, batch.inputs, batch.labels)
    assert abs(float(m[0] / m[1]) - float(ref_loss)) < 2e-2
    for n, g in ref_g.items():
        assert _rel(P.g(n), g) < 6e-2, (n, _rel(P.g(n), g))


def test_stage_split_equals_full_model():
    """Running the stages back to back (activation hand-off, dx chaining) gives the
    same grads as the un-split model."""
    full = TransformerLM(CFG)
    P = FlatParams(full.param_specs()).init_(0)
    batch = lm_batch(CFG, global_batch=2, seed=4)
    loss_and_grad(full, P, batch.inputs, batch.labels, train=False, seed=0, offset=0, step=None)
    stages = [lm_stage(CFG, 2, s) for s in range(2)]
    Ps = []
    for st in stages:
        Q = FlatParams(st.param_specs())
        for n in Q.names():
            Q.p(n).copy_(P.p(n))
        Q.sync_shadow()
        Ps.append(Q)
    h, c0 = stages[0].forward(Ps[0], batch.inputs)
    logits, c1 = stages[1].forward(Ps[1], h)
    from jax_distributed_tuts_amd.ops import kernels as K

    y = batch.labels.reshape(-1)
    dl = torch.empty_like(logits)
    K.softmax_xent(logits, y, grad_scale=1 / y.numel(), dlogits=dl, dbias=Ps[1].g("head/bias"))
    dx = stages[1].backward(Ps[1], c1, dl, need_dx=True)
    stages[0].backward(Ps[0], c0, dx, dout_is_dz=False)
    for Q in Ps:
        for n in Q.names():
            torch.testing.assert_close(Q.g(n), P.g(n), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mode", ["defer", "per-mb", "layer-major"])
def test_deferred_weight_grads_equal_microbatch_loop(mode, monkeypatch):
    """One-stage GPipe step of the LM with per-microbatch passes: the deferred W pass
    (WGradArena: every weight gradient one GEMM over all microbatches' rows after the
    backward chain) == the per-microbatch weight-gradient accumulation == the
    layer-major single pass (one plain-SGD step, lr 1: the applied gradient)."""
    from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline
    from jax_distributed_tuts_amd.utils.train_state import sgd

    def run(defer, layer_major):
        monkeypatch.setenv("JDT_DEFER_WGRAD", "1" if defer else "0")
        tr, _ = build_lm_pipeline(None, "cpu", CFG, num_microbatches=4, tx=sgd(1.0),
                                  layer_major_single_stage=layer_major)
        assert (getattr(tr, "_arena", None) is None)
        before = {k: v.clone() for k, v in tr.state.params.state_dict().items()}
        tr.step(lm_batch(CFG, global_batch=8, seed=7))
        assert (getattr(tr, "_arena", None) is not None) == (defer and not layer_major)
        return {k: before[k] - v for k, v in tr.state.params.state_dict().items()}

    ref = run(False, False)
    got = run(mode == "defer", mode == "layer-major")
    for k in ref:
        torch.testing.assert_close(got[k], ref[k], rtol=2e-4, atol=2e-6, msg=lambda m: f"{k}: {m}")
