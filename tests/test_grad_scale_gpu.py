"""Scale-sensitive GPU checks of the hand-written kernels against the float64
autograd oracle (tests/oracle.py).

* ``mlp2_bwd`` / ``md_bwd`` mode 0 (the raw gradient bucket the N > 1 paths
  all-reduce): P.grad / n_minibatches vs the oracle, dropout ON with the
  kernels' own Philox masks mirrored on the CPU, at the per-GPU row counts of
  N = 1 / 4 / 8 (128 / 32 / 16 rows).
* mode 1 (AdamW fused into the backward epilogue) with eps = 10: the update
  ``g / (|g| + 10)`` is proportional to the gradient (unlike Adam at eps 1e-8),
  so its internal 1/n_minibatch scale is checked too; the gradient is recovered
  exactly as g = 10 d / (1 - |d|).
* the generic per-minibatch GEMM path and the SGD kernel (with/without momentum).
* DP / FSDP / GPipe / DP x PP over the xGMI kernels (processes sharing the GPU):
  the applied gradient of one plain-SGD step (and of the fused xGMI AdamW with
  eps = 10) vs the oracle on the global batch.
"""
import functools
import os

import pytest
import torch

from .gpu_spawn import spawn8
from .oracle import check_grad, mlp_grads_fp64, sgd_grads

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _batch(rows=128):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.utils.config import dp_config

    b = synthetic_batch(dp_config(), 70)
    return b.slice(0, rows)


def _masks(seed, n_hidden, rows, n_mb, H=512, keep=0.9, step=0):
    """Fused-engine masks: layer l over ALL local rows, stream (seed, (l << 1) + (step << 32))."""
    from jax_distributed_tuts_amd.ops.kernels import dropout_mask

    full = [dropout_mask(seed, (l << 1) + (step << 32), (rows, H), keep) for l in range(n_hidden)]
    mb = rows // n_mb
    return [[m[i * mb:(i + 1) * mb] for m in full] + [None] for i in range(n_mb)]


def _state(num_layers, tx, dropout=0.1):
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import init_dp

    return init_dp(Classifier(dropout_rate=dropout, num_layers=num_layers), tx, 69, DEV)


def _cpu(d):
    return {k: v.detach().float().cpu().clone() for k, v in d.items()}


@pytest.mark.parametrize("num_layers", [2, 4])
@pytest.mark.parametrize("rows", [16, 32, 128])
def test_fused_mode0_grads_match_fp64(num_layers, rows):
    from jax_distributed_tuts_amd.parallel.dp import fold_rng_over_axis
    from jax_distributed_tuts_amd.parallel.fused_mlp import make_engine
    from jax_distributed_tuts_amd.utils.flat import N_METRIC_SLOTS
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    st = _state(num_layers, adamw(1e-3))
    b = _batch(rows)
    bg = Batch(b.inputs.to(DEV), b.labels.to(DEV))
    metrics = torch.zeros(N_METRIC_SLOTS, device=DEV)
    eng = make_engine(st, None, "data", 4, rows, metrics, DEV, fuse_opt=False)
    assert eng is not None and not eng.fuse_opt
    P = st.params
    before = _cpu(P.state_dict())
    eng.forward_backward(bg)
    torch.cuda.synchronize()
    got = {n: (P.g(n) / 4).cpu() for n in P.names()}
    seed = fold_rng_over_axis(st.rng, None, "data") & 0xFFFFFFFF
    model = st.apply_fn
    want = mlp_grads_fp64(before, model.names, b.inputs, b.labels,
                          masks=_masks(seed, model.L - 1, rows, 4), keep=0.9, n_mb=4)
    for n in P.names():
        check_grad(got[n], want[n], n)
    # metric slots: loss sum and counts of this step's rows
    slot = P.metrics_slot.cpu()
    assert float(slot[1]) == rows and float(slot[3]) == rows


@pytest.mark.parametrize("num_layers", [2, 4])
def test_fused_mode1_adamw_scale_matches_fp64(num_layers):
    """AdamW inside the backward epilogue (one GPU), eps = 10, weight decay 0."""
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, fold_rng_over_axis
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    st = _state(num_layers, adamw(1.0, eps=10.0, weight_decay=0.0))
    b = _batch()
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    before = _cpu(st.params.state_dict())
    tr.step(Batch(b.inputs.to(DEV), b.labels.to(DEV)))
    tr.finalize()
    torch.cuda.synchronize()
    assert tr.fused is not None and tr.fused.fuse_opt
    after = _cpu(st.params.state_dict())
    seed = fold_rng_over_axis(st.rng, None, "data") & 0xFFFFFFFF
    model = st.apply_fn
    want = mlp_grads_fp64(before, model.names, b.inputs, b.labels, masks=_masks(seed, model.L - 1, 128, 4),
                          keep=0.9, n_mb=4)
    for n in want:
        d = before[n].double() - after[n].double()
        check_grad(10 * d / (1 - d.abs()), want[n], n)


def _adam_inv(before, after):
    """Gradient recovered from one AdamW(b1 = b2 = 0, eps = 10, wd = 0, lr = 1) update:
    d = g / (|g| + 10)  ->  g = 10 d / (1 - |d|)."""
    d = before.double() - after.double()
    return 10 * d / (1 - d.abs())


@pytest.mark.parametrize("num_layers", [2, 4])
def test_run_ahead_adamw_scale_matches_fp64(num_layers):
    """The run-ahead schedule (one launch per step: step t's CE / backward / AdamW + step
    t+1's forward) through its hipGraphs, scale-checked: AdamW with b1 = b2 = 0 and
    eps = 10 makes every step's update g / (|g| + 10), proportional to that step's
    gradient.  The cold graph (step 0: forward + run-ahead backward), the primed graph
    (step 1: its forward already ran inside step 0's launch, with the updated weights)
    and the primed 4-step graph (the total displacement of 4 steps against the fp64
    oracle iterated on the CPU with the kernels' dropout masks)."""
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, fold_rng_over_axis
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    st = _state(num_layers, adamw(1.0, b1=0.0, b2=0.0, eps=10.0, weight_decay=0.0))
    b = _batch()
    bg = Batch(b.inputs.to(DEV), b.labels.to(DEV))
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    tr.step(bg)   # eager step 0 builds the fused engine
    tr.capture(bg, steps_per_graph=4)
    assert tr._ahead is not None, "run-ahead graphs not built"
    seed = fold_rng_over_axis(st.rng, None, "data") & 0xFFFFFFFF
    model = st.apply_fn

    def oracle(params, step):
        return mlp_grads_fp64(params, model.names, b.inputs, b.labels,
                              masks=_masks(seed, model.L - 1, 128, 4, step=step), keep=0.9, n_mb=4)

    # cold replay (step 1) and primed replay (step 2)
    for step in (1, 2):
        before = _cpu(st.params.state_dict())
        tr.step(bg)
        torch.cuda.synchronize()
        after = _cpu(st.params.state_dict())
        want = oracle(before, step)
        for n in want:
            check_grad(_adam_inv(before[n], after[n]), want[n], f"step {step} {n}")
    # primed 4-step graph: steps 3..6 against the iterated fp64 oracle
    before = _cpu(st.params.state_dict())
    tr.run_steps(bg, 4)
    tr.finalize()
    torch.cuda.synchronize()
    after = _cpu(st.params.state_dict())
    p = {n: v.double() for n, v in before.items()}
    for step in range(3, 7):
        g = oracle({n: v.float() for n, v in p.items()}, step)
        for n in g:
            p[n] = p[n] - g[n] / (g[n].abs() + 10.0)
    for n in p:
        check_grad(before[n].double() - after[n].double(), before[n].double() - p[n], f"4 steps {n}")


@pytest.mark.parametrize("accum,streams", [("loop", 1), ("loop", 2), ("loop", 4), ("fused", 1)])
def test_generic_gemm_path_sgd_matches_fp64(accum, streams):
    """Per-minibatch kernels (loop: the fused per-layer md kernels, minibatch i on
    stream i % streams with its own grad set) or generic kernels (fused) + the SGD
    kernel; loop: minibatch i of step 0 draws its masks from (seed, (l << 1) + (i << 32))
    over its own [32, H] block."""
    from jax_distributed_tuts_amd.ops.kernels import dropout_mask
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, fold_rng_over_axis
    from jax_distributed_tuts_amd.utils.train_state import Batch, sgd

    st = _state(2, sgd(1.0))
    b = _batch()
    tr = DataParallelTrainer(st, None, DPConfig(4, accum, loop_streams=streams))
    before = _cpu(st.params.state_dict())
    tr.step(Batch(b.inputs.to(DEV), b.labels.to(DEV)))
    torch.cuda.synchronize()
    seed = fold_rng_over_axis(st.rng, None, "data") & 0xFFFFFFFF
    if accum == "loop":
        masks = [[dropout_mask(seed, i << 32, (32, 512), 0.9), None] for i in range(4)]
    else:
        masks = _masks(seed, 1, 128, 4)
    want = mlp_grads_fp64(before, ["input_dense", "output_dense"], b.inputs, b.labels, masks=masks, keep=0.9, n_mb=4)
    got = sgd_grads(before, _cpu(st.params.state_dict()))
    for n in want:
        check_grad(got[n], want[n], n)
    if accum == "loop":
        assert tr._loop_engine is not None and tr._loop_engine.n_sets == streams
        assert float(st.params.grad.abs().max()) == 0.0   # private sets merged, everything re-zeroed
        assert all(float(g.abs().max()) == 0.0 for g in tr._loop_engine.gx)


@pytest.mark.parametrize("layers", [2, 4])
def test_loop_streams_captured_matches_one_stream(layers):
    """The DP minibatch loop on 2 streams, captured into a multi-step hipGraph, trains
    like the 1-stream eager loop (4 SGD steps; fp32 accumulation order is the only
    difference: the two grad sets are summed after the join)."""
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig
    from jax_distributed_tuts_amd.utils.train_state import Batch, sgd

    res = []
    for streams, cap in ((1, False), (2, True)):
        st = _state(layers, sgd(0.5))
        b = _batch()
        b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
        p0 = st.params.master.clone()
        tr = DataParallelTrainer(st, None, DPConfig(4, "loop", loop_streams=streams))
        if cap:
            tr.step(b)
            tr.capture(b, steps_per_graph=3)
            tr.run_steps(b, 3)
        else:
            for _ in range(4):
                tr.step(b)
        torch.cuda.synchronize()
        res.append(st.params.master - p0)
    rel = float((res[1] - res[0]).norm() / res[0].norm())
    print(f"[loop streams, {layers} layers] update rel diff {rel:.2e}")
    assert rel < 5e-3, rel


@pytest.mark.parametrize("momentum,wd", [(0.0, 0.0), (0.9, 0.0), (0.9, 1e-2)])
def test_sgd_kernel_matches_torch(momentum, wd):
    from jax_distributed_tuts_amd.ops import kernels as K

    n = 100_003
    g = torch.Generator().manual_seed(3)
    p0, gr0 = torch.randn(n, generator=g), torch.randn(n, generator=g)
    p, gr = p0.to(DEV), gr0.to(DEV)
    buf = torch.zeros(n, device=DEV) if momentum else None
    sh = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    ticket = torch.zeros(1, dtype=torch.int32, device=DEV)
    pr, br = p0.double().clone(), torch.zeros(n, dtype=torch.float64)
    for it in range(3):
        K.sgd_step(p, gr, buf, sh, lr=0.1, momentum=momentum, wd=wd, grad_scale=0.25, step=step, ticket=ticket,
                   zero_grad=False)
        d = gr0.double() * 0.25 + wd * pr
        if momentum:
            br = momentum * br + d
            d = br
        pr -= 0.1 * d
    torch.cuda.synchronize()
    torch.testing.assert_close(p.cpu().double(), pr, rtol=1e-5, atol=1e-6)
    assert torch.equal(sh, p.to(torch.bfloat16))
    assert int(step.item()) == 3 and int(ticket.item()) == 0
    # zero_grad=True clears the gradient buffer
    K.sgd_step(p, gr, buf, sh, lr=0.1, momentum=momentum, wd=wd, step=step, ticket=ticket, zero_grad=True)
    torch.cuda.synchronize()
    assert not bool(gr.any())


# ----------------------------------------------------------------------------- over xGMI (shared GPU)
def _load(d, name, ws):
    return [torch.load(os.path.join(d, f"{name}_r{r}.pt"), weights_only=True) for r in range(ws)]


@pytest.mark.parametrize("kind,ws", [("dp_sgd", 2), ("dp_adam_eps", 2), ("dp4_adam_eps", 2), ("fsdp_sgd", 2),
                                     ("fsdp_loop_sgd", 2), ("fsdp_loop_sgd", 4), ("dp_sgd", 8), ("dp_adam_eps", 8),
                                     ("dp4_adam_eps", 8), ("fsdp_sgd", 8), ("fsdp_loop_sgd", 8),
                                     ("fsdp4_adam_eps", 2), ("fsdp4_adam_eps", 8)])
def test_xgmi_strategies_grad_scale(tmp_path, kind, ws):
    """dp4_adam_eps at ws = 2: the 4-layer DP step with every hidden layer's backward
    exchanging its tiles in-kernel (AdamW eps = 10: the update is ~ the gradient);
    at ws = 8 (8 grids do not fit one GPU): the xGMI all-reduce + AdamW step."""
    from jax_distributed_tuts_amd.runtime.launch import spawn

    from . import xgmi_workers as XW

    spawn(functools.partial(XW.grad_probe_xgmi, kind=kind), ws, str(tmp_path), gpu=True)
    res = _load(tmp_path, f"gpx_{kind}", ws)
    assert all(o["comm"] == "xgmi" for o in res)
    b = _batch()
    deep = kind in ("dp4_adam_eps", "fsdp4_adam_eps")
    names = (["input_dense", "hidden_dense_1", "hidden_dense_2", "output_dense"] if deep
             else ["input_dense", "output_dense"])
    if kind == "fsdp4_adam_eps":
        # 2 ranks: the in-kernel owner exchange (no step collective)
        assert all(o["one_launch"] == (ws == 2) for o in res), [o["one_launch"] for o in res]
    want = mlp_grads_fp64(res[0]["before"], names, b.inputs, b.labels, n_mb=4)
    for o in res:
        for n in want:
            d = o["before"][n].double() - o["after"][n].double()
            g = 10 * d / (1 - d.abs()) if kind.endswith("adam_eps") else d
            check_grad(g, want[n], n)


@pytest.mark.parametrize("ws", [2, 4, 8])
def test_pipeline_stage_kernel_adam_scale(tmp_path, ws, monkeypatch):
    """One layer per stage, AdamW eps = 10 (update ~ gradient): each stage's step is the
    in-kernel GPipe launch (ops/csrc/pp_stage.hip: dZ hops, dH from the successor's weight
    image, register-held dW, AdamW at the end) -- its update equals the fp64 oracle's.
    ws = 8: BASELINE config #4's 8-stage layout, the 8 ranks' stage grids filling the one
    GPU's 256 CUs (JDT_PP_STAGE_SPARE=0 lifts the half-free rule for ranks sharing it)."""
    if ws == 8:
        monkeypatch.setenv("JDT_PP_STAGE_SPARE", "0")
    from pipeline_parallel import pp_mlp_dims
    from jax_distributed_tuts_amd.models.mlp import MLP
    from jax_distributed_tuts_amd.utils.config import dp_config

    from . import xgmi_workers as XW

    spawn8(functools.partial(XW.grad_probe_xgmi, kind="pp_adam_eps", dp=1, n_hidden=ws), ws, str(tmp_path))
    res = _load(tmp_path, "gpx_pp_adam_eps", ws)
    assert all(o["comm"] == "xgmi" and o["pp_kernel"] for o in res), [(o["comm"], o["pp_kernel"]) for o in res]
    before, got = {}, {}
    for o in res:
        before.update(o["before"])
        for k in o["before"]:
            d = o["before"][k].double() - o["after"][k].double()
            got[k] = 10 * d / (1 - d.abs())
    b = _batch()
    want = mlp_grads_fp64(before, MLP(pp_mlp_dims(dp_config(), ws)).names, b.inputs, b.labels, n_mb=4)
    assert set(got) == set(want)
    for n in want:
        check_grad(got[n], want[n], n)


@pytest.mark.parametrize("ws,dp,n_hidden", [(2, 1, 3), (4, 2, 3), (8, 1, 7), (8, 2, 3)])
def test_xgmi_pipeline_grad_scale(tmp_path, ws, dp, n_hidden):
    from pipeline_parallel import pp_mlp_dims
    from jax_distributed_tuts_amd.models.mlp import MLP
    from jax_distributed_tuts_amd.runtime.launch import spawn
    from jax_distributed_tuts_amd.utils.config import dp_config

    from . import xgmi_workers as XW

    spawn8(functools.partial(XW.grad_probe_xgmi, kind="pp_sgd", dp=dp, n_hidden=n_hidden), ws, str(tmp_path))
    res = _load(tmp_path, "gpx_pp_sgd", ws)
    before, got = {}, {}
    for o in res:
        assert o["comm"] == "xgmi"
        before.update(o["before"])
        for k, v in sgd_grads(o["before"], o["after"]).items():
            if k in got:
                torch.testing.assert_close(v, got[k], rtol=0, atol=0)
            got[k] = v
    b = _batch()
    want = mlp_grads_fp64(before, MLP(pp_mlp_dims(dp_config(), n_hidden)).names, b.inputs, b.labels, n_mb=4)
    assert set(got) == set(want)
    for n in want:
        check_grad(got[n], want[n], n)
