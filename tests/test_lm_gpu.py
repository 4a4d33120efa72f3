"""Transformer LM on the GPU at the BENCH configuration (4 layers, d 512, 8 heads,
d_ff 2048, S 128, V 2048, 16 sequences, 4 microbatches): every leaf's applied
gradient against a float64 autograd oracle, and the in-epilogue AdamW
(ops.kernels.EpilogueAdamW) against the plain AdamW pass."""
import os

import pytest
import torch

from jax_distributed_tuts_amd.models.transformer import TransformerConfig
from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline, lm_batch
from jax_distributed_tuts_amd.utils.train_state import Batch, adamw, sgd

from .oracle import check_grad, lm_grads_fp64, sgd_grads

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CFG = TransformerConfig()   # the bench model


def _trainer(tx, layer_major=True, fused_opt="1", wpass=None):
    old = os.environ.get("JDT_LM_FUSED_OPT")
    os.environ["JDT_LM_FUSED_OPT"] = fused_opt
    try:
        tr, _ = build_lm_pipeline(None, DEV, CFG, num_microbatches=4, tx=tx, layer_major_single_stage=layer_major,
                                  mb_streams=1 if layer_major else None, wpass_streams=wpass)
        b = lm_batch(CFG, global_batch=16, seed=1)
        b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
        tr.step(b)   # builds the epilogue optimizer (env read here)
    finally:
        if old is None:
            os.environ.pop("JDT_LM_FUSED_OPT", None)
        else:
            os.environ["JDT_LM_FUSED_OPT"] = old
    return tr, b


@pytest.mark.parametrize("layer_major,streams,early", [(True, 1, 0), (True, 3, 0), (False, 1, 0), (False, 2, 0),
                                                      (False, 4, 0), (False, 4, 2)])
def test_lm_bench_config_grads_match_fp64_autograd(layer_major, streams, early):
    """One plain-SGD (lr 1) step: p_before - p_after is the applied gradient (mean CE
    over all 2048 tokens); every one of the 54 leaves within the pinned oracle
    tolerance (bf16 operands).  Per-microbatch passes: microbatch i on stream
    i % streams; layer-major: the deferred weight-gradient GEMMs on streams - 1 side
    streams, overlapping the input-gradient chain."""
    tr0, _ = build_lm_pipeline(None, DEV, CFG, num_microbatches=4, tx=sgd(1.0), layer_major_single_stage=layer_major,
                               mb_streams=1 if layer_major else streams, wpass_streams=streams)
    assert tr0.single_stage_mode == ("layer-major" if layer_major else
                                     f"microbatch-loop ({streams} streams)" if streams > 1 else "microbatch-loop")
    tr0.cfg.wpass_early = early   # > 0: the W pass on its own streams, per part as the chains pass it
    before = {k: v.detach().clone() for k, v in tr0.state.params.state_dict().items()}
    bb = lm_batch(CFG, global_batch=16, seed=1)
    tr0.step(Batch(bb.inputs.to(DEV), bb.labels.to(DEV)))
    torch.cuda.synchronize()
    got = sgd_grads(before, tr0.state.params.state_dict())
    want = lm_grads_fp64({k: v.to(DEV) for k, v in before.items()}, CFG, bb.inputs.to(DEV), bb.labels.to(DEV))
    assert set(got) == set(want) and len(got) == 54
    worst = 0.0
    for k in sorted(want):
        rel, scale = check_grad(got[k].cpu(), want[k].cpu(), k, rel_tol=0.025, scale_tol=0.004)  # measured max 0.0126 / 0.0015
        worst = max(worst, rel)
    print(f"[lm bench grads, layer_major={layer_major}, streams={streams}, early={early}] worst rel err {worst:.3e}")


@pytest.mark.parametrize("layer_major,wpass", [(True, 1), (True, 3), (False, None)])
def test_lm_epilogue_adamw_matches_plain_adamw(layer_major, wpass):
    """AdamW fused into the weight-gradient GEMM epilogues (+ one multi-range launch for
    the rest) == the plain full-buffer AdamW pass, after 3 steps; the step counter
    advances once per step.  The step is not bitwise reproducible (fp32 atomics in the
    attention / LayerNorm / embedding / bias reductions; a second plain run shows the
    noise -- layer-major runs usually come out bit-equal, not always), and AdamW turns
    tiny gradient differences into lr-sized updates where g ~ 0 -- so the check is that
    no weight leaf has more than 2 % of its elements half an update apart (a missed
    microbatch contribution or a wrong gradient scale moves most of a leaf), plus the
    loss sums."""
    lr = 3e-4
    res = {}
    for fused in ("1", "0", "0b"):
        tr, b = _trainer(adamw(lr), layer_major, fused[0], wpass)
        assert (getattr(tr, "_eo", None) not in (None, False)) == (fused == "1")
        tr.step(b)
        tr.step(b)
        torch.cuda.synchronize()
        res[fused] = (tr.state.params, tr.state.params.master.clone(), tr.state.params.shadow.clone(),
                      int(tr.state.opt_state["count"].item()), tr.state.params.grad.abs().max().item(),
                      float(tr.metrics[0]))
    (P1, p1, s1, c1, g1, l1), (P0, p0, s0, c0, g0, l0) = res["1"], res["0"]
    assert c1 == c0 == 3
    assert g1 == 0.0 and g0 == 0.0   # gradient buffers left zeroed for the next step
    assert float(((s1.float() - p1.to(torch.bfloat16).float()).abs()).max()) == 0.0   # shadow = bf16(master)
    noise_loss = abs(res["0b"][5] - l0)
    assert abs(l1 - l0) <= 1e-3 * abs(l0) + 4 * noise_loss, (l1, l0, res["0b"][5])
    for n in P0.names():
        a, c = p1[P0.offsets[n][0]:P0.offsets[n][0] + P0.p(n).numel()], p0[P0.offsets[n][0]:P0.offsets[n][0] + P0.p(n).numel()]
        if a.numel() < 4096:
            continue
        frac = float(((a - c).abs() > 0.5 * lr).float().mean())
        nb = res["0b"][1][P0.offsets[n][0]:P0.offsets[n][0] + P0.p(n).numel()]
        noise = float(((nb - c).abs() > 0.5 * lr).float().mean())
        print(f"{n:28s} apart {frac:.2e} (noise {noise:.2e})")
        assert frac <= 0.02 + 4 * noise, (n, frac, noise)


def test_lm_microbatch_streams_captured_matches_eager():
    """Per-microbatch passes on 1 stream (eager) vs 2 streams (eager and hipGraph-captured,
    the fork / join recorded in the graph): 3 SGD steps move the parameters by the same
    amount up to the fp32-atomic reduction-order noise."""
    res = {}
    for streams, cap in ((1, False), (2, False), (2, True), (4, True)):
        tr, _ = build_lm_pipeline(None, DEV, CFG, num_microbatches=4, tx=sgd(0.5), layer_major_single_stage=False,
                                  mb_streams=streams)
        tr.cfg.wpass_early = 2 if streams == 4 else 0
        bb = lm_batch(CFG, global_batch=16, seed=1)
        b = Batch(bb.inputs.to(DEV), bb.labels.to(DEV))
        p0 = tr.state.params.master.clone()
        if cap:
            tr.capture(b)
            tr.run_steps(b, 3)
        else:
            for _ in range(3):
                tr.step(b)
        torch.cuda.synchronize()
        res[(streams, cap)] = tr.state.params.master - p0
        assert int(tr.state.step) == 3
    ref = res[(1, False)]
    for key in ((2, False), (2, True), (4, True)):
        rel = float((res[key] - ref).norm() / ref.norm())
        print(f"[lm mb streams] {key}: update rel diff {rel:.2e}")
        assert rel < 0.02, (key, rel)
