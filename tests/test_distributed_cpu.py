"""T2/T3 on the CPU fake cluster: gloo world of N processes (the analogue of the
reference's sim_multiCPU_dev; BASELINE config #1 is gloo world_size=2)."""
import functools
import os

import pytest
import torch

from jax_distributed_tuts_amd.runtime.launch import spawn

from . import dist_workers as W

pytestmark = pytest.mark.slow


def _adam_close(a, b, lr=1e-3, steps=3, frac=1e-3):
    """Adam normalises each coordinate, so an element whose gradient is ~0 can move
    by up to lr per step from rounding-order noise alone; require that only a tiny
    fraction of elements deviate, and none by more than the Adam step bound."""
    d = (a.float() - b.float()).abs()
    assert float(d.max()) <= 2 * lr * steps + 1e-6, float(d.max())
    assert float((d > 5e-5).float().mean()) < frac


def _metrics_close(m, ref):
    assert abs(float(m[0]) - float(ref[0])) <= 1e-3 * abs(float(ref[0])) + 1e-3
    assert float(m[1]) == float(ref[1]) and float(m[3]) == float(ref[3])
    assert abs(float(m[2]) - float(ref[2])) <= 2  # argmax ties may flip


def _load(d, name, ws):
    return [torch.load(os.path.join(d, f"{name}_r{r}.pt"), weights_only=False) for r in range(ws)]


@pytest.mark.parametrize("ws", [2, 4])
def test_collectives_semantics(tmp_path, ws):
    spawn(W.collectives, ws, str(tmp_path))
    res = _load(tmp_path, "coll", ws)
    xs = [torch.arange(8, dtype=torch.float32) + 100 * r for r in range(ws)]
    tot = sum(xs)
    for r, o in enumerate(res):
        assert o["idx"] == r
        torch.testing.assert_close(o["psum"], tot)
        torch.testing.assert_close(o["pmean"], tot / ws)
        torch.testing.assert_close(o["ag0"], torch.cat([x.view(2, 4) for x in xs], 0))
        torch.testing.assert_close(o["ag1"], torch.cat([x.view(2, 4) for x in xs], 1))
        full = sum(torch.arange(4 * ws, dtype=torch.float32).view(2 * ws, 2) * (q + 1) for q in range(ws))
        torch.testing.assert_close(o["rs"], full[2 * r: 2 * r + 2])
        torch.testing.assert_close(o["ring"], xs[(r - 1) % ws])


def test_mesh_2d_groups(tmp_path):
    spawn(W.mesh2d, 4, str(tmp_path))
    res = _load(tmp_path, "mesh", 4)
    # ("data", "pipe") = (2, 2), row-major: rank = d*2 + p
    for r, o in enumerate(res):
        d, p = divmod(r, 2)
        assert o["coords"] == (d, p)
        assert o["pipe_ranks"] == (2 * d, 2 * d + 1)
        assert o["data_ranks"] == (p, 2 + p)
        assert float(o["pipe_sum"]) == (2 * d) + (2 * d + 1)
        assert float(o["data_sum"]) == p + (2 + p)


def test_gather_arr_mean_grads(tmp_path):
    ws = 2
    spawn(W.gather_mean_grad, ws, str(tmp_path))
    res = _load(tmp_path, "gmg", ws)
    full = torch.cat([torch.arange(6, dtype=torch.float32).view(3, 2) + 10 * r for r in range(ws)], 0)
    wsum = sum(torch.arange(12, dtype=torch.float32).view(6, 2) * (r + 1) for r in range(ws))
    for r, o in enumerate(res):
        torch.testing.assert_close(o["full"], full)
        # backward = reduce-scatter of d(out)/d(full) = w_r summed over ranks, / N
        torch.testing.assert_close(o["grad"], (wsum / ws)[3 * r: 3 * r + 3])


def _single_device_reference(steps=3, accum="loop"):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import adamw

    model = Classifier(dropout_rate=0.0)
    st = init_dp(model, adamw(1e-3), 69, "cpu")
    tr = DataParallelTrainer(st, None, DPConfig(4, accum))
    b = synthetic_batch(dp_config(), 70)
    for _ in range(steps):
        tr.step(b)
    return st.params.state_dict(), tr.metrics


@pytest.mark.parametrize("accum", ["loop", "scan", "fused"])
def test_dp2_equals_single_device(tmp_path, accum):
    """DP over 2 ranks (each 2 minibatches of 16 rows... i.e. 64 rows/rank) must equal
    single-device training on the same global batch when dropout is off: the
    per-minibatch row sets differ, but every row carries weight 1/128 either way."""
    spawn(functools.partial(W.dp_vs_single, accum=accum), 2, str(tmp_path))
    res = _load(tmp_path, f"dp_{accum}", 2)
    ref_p, ref_m = _single_device_reference(accum=accum)
    for o in res:
        for k in ref_p:
            _adam_close(o["params"][k], ref_p[k])
        _metrics_close(o["metrics"], ref_m)
    torch.testing.assert_close(res[0]["params"]["input_dense/kernel"], res[1]["params"]["input_dense/kernel"],
                               rtol=0, atol=0)


@pytest.mark.parametrize("gather_once", [False, True])
def test_fsdp2_equals_single_device(tmp_path, gather_once):
    spawn(functools.partial(W.fsdp_run, gather_once=gather_once), 2, str(tmp_path))
    res = _load(tmp_path, f"fsdp_{int(gather_once)}", 2)
    ref_p, ref_m = _single_device_reference()
    for o in res:
        for k in ref_p:
            _adam_close(o["params"][k], ref_p[k])
        _metrics_close(o["metrics"], ref_m)


def test_shard_module_params_autograd(tmp_path):
    ws = 2
    spawn(W.sharded_module, ws, str(tmp_path))
    res = _load(tmp_path, "sm", ws)
    net = torch.nn.Sequential(torch.nn.Linear(16, 8), torch.nn.Tanh(), torch.nn.Linear(8, 4))
    net.load_state_dict(res[0]["ref"])
    loss = 0
    for o in res:
        out = net(o["x"])
        torch.testing.assert_close(o["out"], out.detach(), rtol=1e-5, atol=1e-6)
        loss = loss + out.square().mean()
    (loss / ws).backward()  # DP-mean of the per-rank losses
    full_grads = {n: p.grad for n, p in net.named_parameters()}
    for r, o in enumerate(res):
        for n, g in o["grads"].items():
            if n in o["meta"]:
                d = o["meta"][n][0].index("data")
                exp = full_grads[n].chunk(ws, dim=d)[r]
            else:
                exp = full_grads[n]
            torch.testing.assert_close(g, exp, rtol=1e-4, atol=1e-6)


def _single_mlp_reference(n_hidden=3, steps=3, n_mb=4):
    from data_paral import synthetic_batch
    from pipeline_parallel import pp_mlp_dims
    from jax_distributed_tuts_amd.models.mlp import MLP
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.flat import FlatParams
    from jax_distributed_tuts_amd.utils.train_state import TrainState, adamw
    from jax_distributed_tuts_amd.utils import rng as R

    cfg = dp_config()
    model = MLP(pp_mlp_dims(cfg, n_hidden), dropout_rate=0.0)
    P = FlatParams(model.param_specs()).init_(cfg.seed)
    st = TrainState.create(apply_fn=model, params=P, tx=adamw(1e-3), rng=R.PRNGKey(cfg.seed))
    tr = DataParallelTrainer(st, None, DPConfig(n_mb, "loop"))
    b = synthetic_batch(cfg, 70)
    for _ in range(steps):
        tr.step(b)
    return P.state_dict(), tr.metrics


@pytest.mark.parametrize("ws,dp", [(2, 1), (4, 1), (4, 2)])
def test_pipeline_equals_single_device(tmp_path, ws, dp):
    """GPipe over S stages (and hybrid DP x PP) == the un-split model on one device
    (dropout off): per-stage params match the corresponding slice."""
    spawn(functools.partial(W.pp_run, dp=dp), ws, str(tmp_path))
    res = _load(tmp_path, f"pp_dp{dp}", ws)
    ref_p, ref_m = _single_mlp_reference()
    seen = set()
    for o in res:
        for k, v in o["params"].items():
            # a stage boundary rounds dh to bf16 before act' (the fused single-device
            # epilogue rounds once), so allow a few % of Adam-amplified coordinates
            _adam_close(v, ref_p[k], frac=5e-2)
            seen.add(k)
        _metrics_close(o["metrics"], ref_m)
    assert seen == set(ref_p)


def test_replication_checker(tmp_path):
    spawn(W.replication, 2, str(tmp_path))
    for o in _load(tmp_path, "rep", 2):
        assert "diverged" in o["res"] and "'w'" in o["res"]


def test_checkpoint_resume_fsdp(tmp_path):
    """save after 2 steps, restore into a fresh sharded state, step once ==
    uninterrupted 3 steps (rank-local safetensors shards)."""
    spawn(W.ckpt, 2, str(tmp_path))
    for o in _load(tmp_path, "ck", 2):
        assert o["step"] == 3 and o["count"] == 3
        for k in o["ref"]:
            torch.testing.assert_close(o["got"][k], o["ref"][k], rtol=0, atol=0)


def test_bucketed_overlap_equals_single_allreduce(tmp_path):
    """Async bucketed all-reduce fired from backward(on_ready) == one whole-buffer all-reduce."""
    spawn(functools.partial(W.dp_overlap, overlap=True, bucket_mb=0.5), 2, str(tmp_path))
    spawn(functools.partial(W.dp_overlap, overlap=False, bucket_mb=0.5), 2, str(tmp_path))
    a, b = _load(tmp_path, "ov1", 2), _load(tmp_path, "ov0", 2)
    assert a[0]["nb"] >= 3  # several buckets for the 4-layer MLP at 0.5 MiB
    for x, y in zip(a, b):
        for k in x["params"]:
            torch.testing.assert_close(x["params"][k], y["params"][k], rtol=0, atol=0)
        torch.testing.assert_close(x["metrics"], y["metrics"], rtol=0, atol=0)


@pytest.mark.parametrize("mode", ["loop", "merged", "layer-major"])
def test_single_stage_pipeline_merge_equals_reference(mode):
    """A one-stage GPipe step -- microbatch loop, merged into one pass
    (PipeConfig.merge_single_stage), or layer-major (the default for a model without
    dropout) -- == single-device accumulation (dropout off)."""
    from data_paral import synthetic_batch
    from pipeline_parallel import pp_mlp_dims
    from jax_distributed_tuts_amd.models.mlp import MLP
    from jax_distributed_tuts_amd.parallel.pipeline import GPipeTrainer, PipeConfig, init_stage_params, mlp_stage
    from jax_distributed_tuts_amd.utils import rng as R
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import TrainState, adamw

    cfg = dp_config()
    dims = pp_mlp_dims(cfg, 3)
    stage = mlp_stage(dims, 1, 0, dropout_rate=0.0)
    P = init_stage_params(stage, MLP(dims, dropout_rate=0.0).param_specs(), cfg.seed, "cpu")
    st = TrainState.create(apply_fn=stage, params=P, tx=adamw(1e-3), rng=R.PRNGKey(cfg.seed))
    tr = GPipeTrainer(st, None, PipeConfig(4, merge_single_stage=mode == "merged",
                                           layer_major_single_stage=mode != "loop"))
    assert tr.single_stage_mode == ("microbatch-loop" if mode == "loop" else mode)
    b = synthetic_batch(cfg, 70)
    for _ in range(3):
        tr.step(b)
    ref_p, ref_m = _single_mlp_reference()
    for k, v in P.state_dict().items():
        _adam_close(v, ref_p[k], frac=5e-2)
    _metrics_close(tr.metrics, ref_m)
