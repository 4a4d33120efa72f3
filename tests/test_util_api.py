"""T0: util.py API parity (reference util.py:1-185)."""
import math

import pytest
import torch

import util
from jax_distributed_tuts_amd.models.mlp import Classifier
from jax_distributed_tuts_amd.utils import rng as R
from jax_distributed_tuts_amd.utils.flat import FlatParams


def test_print_metrics_golden(capsys):
    util.print_metrics({"loss": (torch.tensor(3.0), torch.tensor(2.0)), "accuracy": (5, 8)}, "dp")
    out = capsys.readouterr().out
    assert out == "======= dp =======\nloss: 1.500000\naccuracy: 0.625000\n"
    util.print_metrics(torch.tensor([1.0, 4.0, 2.0, 4.0]), "")
    assert capsys.readouterr().out == "loss: 0.250000\naccuracy: 0.500000\n"


def test_print_exception(capsys):
    util.print_exception(ValueError("boom"))
    out = capsys.readouterr().out
    assert "ValueError" in out and "boom" in out


def test_batch_slice_and_map():
    b = util.Batch(torch.arange(12.0).view(6, 2), torch.arange(6, dtype=torch.int32))
    s = b.slice(2, 3)
    assert s.inputs.shape == (3, 2) and s.labels.tolist() == [2, 3, 4]
    m = b.map(lambda t: t[:1])
    assert m.size == 1


def test_num_params_reference_model():
    model = Classifier()
    P = FlatParams(model.param_specs())
    st = util.TrainState.create(apply_fn=model, params=P, tx=util.adamw(1e-3), rng=0)
    assert util.get_num_params(st) == 407050 == 784 * 512 + 512 + 512 * 10 + 10
    names = [s.name for s in model.param_specs()]
    assert names == ["input_dense/kernel", "input_dense/bias", "output_dense/kernel", "output_dense/bias"]
    assert P.p("input_dense/kernel").shape == (784, 512)


def test_lecun_init_statistics():
    P = FlatParams(Classifier().param_specs()).init_(0)
    w = P.p("input_dense/kernel")
    assert abs(float(w.std()) - math.sqrt(1 / 784)) < 0.1 * math.sqrt(1 / 784)
    assert float(w.abs().max()) <= 2.0 * math.sqrt(1 / 784) / 0.8796 + 1e-6
    assert float(P.p("input_dense/bias").abs().max()) == 0.0
    assert torch.equal(P.shadow[: P.numel].float(), P.master[: P.numel].to(torch.bfloat16).float())


def test_rng_fold_split_deterministic():
    k = R.PRNGKey(69)
    assert R.split(k, 4) == R.split(k, 4)
    assert len(set(R.split(k, 4))) == 4
    assert R.fold_in(k, 0) != R.fold_in(k, 1)


def _engine_loss_fn(model):
    from jax_distributed_tuts_amd.models.mlp import loss_and_grad

    def loss_fn(params, apply_fn, batch, rng, minibatch_index=0, state=None):
        m = torch.zeros(4)
        loss_and_grad(apply_fn, params, batch.inputs, batch.labels, train=False, seed=rng & 0xFFFF, offset=0,
                      step=None, grad_scale=1.0 / batch.size, metrics=m)
        return m[0] / m[1], {"loss": (m[0], m[1]), "accuracy": (m[2], m[3])}

    return loss_fn


@pytest.mark.gpu
def test_engine_scan_one_minibatch_repeats():
    """accum_grads(use_scan=True, num_minibatches=1) with an engine loss, called twice:
    the cached entry has no captured graph (nothing to roll), so the second call runs the
    body eagerly -- and both calls equal the unrolled loop."""
    dev = torch.device("cuda", 0)
    model = Classifier(dropout_rate=0.0)
    g = torch.Generator().manual_seed(0)
    x, y = torch.randn(32, 784, generator=g).to(dev), torch.randint(0, 10, (32,), generator=g).to(torch.int32).to(dev)

    def loss_fn(params, apply_fn, batch, rng, minibatch_index=0, state=None):
        from jax_distributed_tuts_amd.models.mlp import loss_and_grad

        m = torch.zeros(4, device=dev)
        loss_and_grad(apply_fn, params, batch.inputs, batch.labels, train=False, seed=rng & 0xFFFF, offset=0,
                      step=None, grad_scale=1.0 / batch.size, metrics=m)
        return m[0] / m[1], {"loss": (m[0], m[1]), "accuracy": (m[2], m[3])}

    P = FlatParams(model.param_specs(), device=dev).init_(1)
    st = util.TrainState.create(apply_fn=model, params=P, tx=util.adamw(1e-3), rng=R.PRNGKey(0))
    util.accum_grads(st, util.Batch(x, y), R.PRNGKey(1), 1, loss_fn, False)
    want = P.grad.clone()
    for _ in range(2):
        P.zero_grad()
        _, m = util.accum_grads(st, util.Batch(x, y), R.PRNGKey(1), 1, loss_fn, True)
        torch.cuda.synchronize()
        assert torch.equal(P.grad, want)
        assert float(m["loss"][1]) == 32.0


@pytest.mark.parametrize("use_scan", [False, True])
def test_accum_grads_matches_full_batch(use_scan):
    """mean over minibatches of minibatch-mean grads == full-batch mean grad (util.py:77)."""
    torch.manual_seed(0)
    model = Classifier(dropout_rate=0.0)
    x, y = torch.randn(32, 784), torch.randint(0, 10, (32,), dtype=torch.int32)
    P = FlatParams(model.param_specs()).init_(1)
    st = util.TrainState.create(apply_fn=model, params=P, tx=util.adamw(1e-3), rng=R.PRNGKey(0))
    grads, metrics = util.accum_grads(st, util.Batch(x, y), R.PRNGKey(1), 4, _engine_loss_fn(model), use_scan)
    g4 = grads.flat * grads.scale
    P.zero_grad()
    grads1, metrics1 = util.accum_grads(st, util.Batch(x, y), R.PRNGKey(1), 1, _engine_loss_fn(model), use_scan)
    torch.testing.assert_close(g4, grads1.flat * grads1.scale, rtol=2e-2, atol=2e-4)
    assert float(metrics["loss"][1]) == 32.0
    torch.testing.assert_close(metrics["loss"][0], metrics1["loss"][0], rtol=1e-4, atol=1e-4)


def test_apply_gradients_adamw_cpu():
    model = Classifier()
    P = FlatParams(model.param_specs()).init_(0)
    st = util.TrainState.create(apply_fn=model, params=P, tx=util.adamw(1e-2), rng=0)
    P.grad[: P.numel].fill_(1.0)
    w0 = P.p("input_dense/kernel").clone()
    st.apply_gradients(grads=util.GradBuffer(P, 0.5))
    # first AdamW step: update = lr * (sign(g) + wd * w)
    exp = w0 - 1e-2 * (1.0 + 1e-4 * w0)
    torch.testing.assert_close(P.p("input_dense/kernel"), exp, rtol=1e-5, atol=1e-6)
    assert st.step == 1 and int(st.opt_state["count"]) == 1
    assert float(P.grad.abs().max()) == 0.0


def test_default_microbatches_follows_measured_table():
    """pipeline.default_microbatches: the count the measured GPipe table picked
    (profiles/r3_pp_schedule.json: best modeled step of the 8-stage MLP at n = 2, the
    4-stage LM within 3 % of its best there); a single stage keeps the tutorial's 4."""
    import json
    import os

    from jax_distributed_tuts_amd.parallel.pipeline import default_microbatches

    assert default_microbatches(1) == 4
    assert all(default_microbatches(s) == 2 for s in (2, 4, 8))
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r3_pp_schedule.json")
    rep = json.load(open(path))
    mlp = rep["layouts"]["mlp_pp8"]
    assert mlp["best_n_mb"] == default_microbatches(mlp["stages"])
    lm = {r["n_mb"]: r["modeled_step_us"] for r in rep["layouts"]["lm_pp4"]["table"]}
    assert lm[default_microbatches(4)] <= 1.05 * min(lm.values())


def test_stream_schedules_resolve_on_cpu(monkeypatch):
    """The concurrent-stream schedules are GPU-only: on CPU a one-stage LM pipeline keeps
    layer-major (or the serial microbatch loop), its stream set is a no-op, and the DP
    loop's auto stream count follows the measured rule (2 for >= 3 layers, else 1)."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.models.transformer import TransformerConfig
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.parallel.pipeline import PipeConfig, _MbStreams
    from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline
    from jax_distributed_tuts_amd.utils.train_state import adamw

    monkeypatch.delenv("JDT_MB_STREAMS", raising=False)
    monkeypatch.delenv("JDT_LOOP_STREAMS", raising=False)
    # mb_streams 0 = auto: 4 streams, or 1 (layer-major) where the one-launch W pass applies (GPU)
    assert PipeConfig().mb_streams == 0 and PipeConfig().wpass_early == 0 and PipeConfig().wpass_rr == 0
    cfg = TransformerConfig(n_layers=1, d_model=64, n_heads=1, d_ff=128, seq_len=16, vocab_size=64)
    for lm, mode in ((True, "layer-major"), (False, "microbatch-loop")):
        tr, _ = build_lm_pipeline(None, "cpu", cfg, num_microbatches=4, layer_major_single_stage=lm)
        assert tr._mb_streams_k() == 1 and tr.single_stage_mode == mode
    on = _MbStreams(None, None)
    on.fork()
    on.join()
    with on(3):
        pass
    for layers, want in ((2, 1), (3, 2), (4, 2)):
        st = init_dp(Classifier(num_layers=layers), adamw(1e-3), 0, "cpu")
        assert DataParallelTrainer(st, None, DPConfig(4, "loop"))._loop_sets() == want
    monkeypatch.setenv("JDT_LOOP_STREAMS", "3")
    st = init_dp(Classifier(num_layers=2), adamw(1e-3), 0, "cpu")
    assert DataParallelTrainer(st, None, DPConfig(4, "loop"))._loop_sets() == 3
