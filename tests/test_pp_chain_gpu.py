"""The one-GPU chain (csrc/pp_stage.hip pp_chain_kernel, parallel/pp_kernel.PPChainKernel):
a one-stage GPipe of the 784 -> 512 x L -> 10 MLP runs every hidden layer as a stage of
ONE launch (32 workgroups each, local inboxes), then one AdamW launch.

* equal to the one-stage path it replaces (the layer-by-layer md kernels with
  per-microbatch dropout streams), dropout ON, eager + captured steps;
  (opt-in, JDT_PP_CHAIN=1: slower than that path, BENCH_NOTES round 5)
* its AdamW(eps = 10) update against the fp64 autograd oracle (update ~ gradient)."""
import os

import pytest
import torch

from .oracle import check_grad, mlp_grads_fp64

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _build(L, n_mb, dropout, tx=None, kernel="1"):
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch

    os.environ["JDT_PP_CHAIN"] = kernel
    try:
        cfg = dp_config()
        tr = build_mlp_pipeline(cfg, Mesh({"data": 1, "pipe": 1}), DEV, n_hidden_layers=L, dropout_rate=dropout,
                                num_microbatches=n_mb, tx=tx)
        b = synthetic_batch(cfg, 70)
        b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
        tr.step(b)   # the engine is chosen here
    finally:
        os.environ.pop("JDT_PP_CHAIN", None)
    return tr, b


@pytest.mark.parametrize("L,n_mb", [(2, 4), (3, 2), (8, 4), (8, 2)])
def test_chain_equals_layer_by_layer(L, n_mb):
    runs = {}
    for k in ("1", "0"):
        tr, b = _build(L, n_mb, 0.1, kernel=k)
        assert (tr.pp_kernel is not None) == (k == "1")
        tr.capture(b, steps_per_graph=2)
        tr.run_steps(b, 3)
        torch.cuda.synchronize()
        tr.finalize()
        runs[k] = ({n: v.detach().float().cpu() for n, v in tr.state.params.state_dict().items()},
                   tr.gather_metrics().cpu(), int(tr.state.step_tensor.item()))
    (pa, ma, ca), (pb, mb_, cb) = runs["1"], runs["0"]
    assert ca == cb == 4
    # AdamW moves an element whose bf16-rounded gradient flips sign by up to 2 lr a step;
    # the share of such elements grows with the depth the gradient crossed (both paths
    # round every activation / dZ to bf16, in different summation orders)
    frac = 2e-2 if L <= 4 else 5e-2
    for n, v in pa.items():
        d = (v - pb[n]).abs()
        assert float(d.max()) <= 2 * 1e-3 * 4 + 1e-6, n
        assert float((d > 5e-5).float().mean()) < frac, (n, float((d > 5e-5).float().mean()))
    assert float(ma[1]) == float(mb_[1]) and abs(float(ma[0]) - float(mb_[0])) <= 2e-3 * abs(float(mb_[0])) + 1e-2
    assert abs(float(ma[2]) - float(mb_[2])) <= 2


@pytest.mark.parametrize("L", [2, 8])
def test_chain_adam_scale_matches_fp64(L):
    from pipeline_parallel import pp_mlp_dims
    from jax_distributed_tuts_amd.models.mlp import MLP
    from jax_distributed_tuts_amd.utils.config import dp_config
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    os.environ["JDT_PP_CHAIN"] = "1"
    try:
        cfg = dp_config()
        tr = build_mlp_pipeline(cfg, Mesh({"data": 1, "pipe": 1}), DEV, n_hidden_layers=L, dropout_rate=0.0,
                                num_microbatches=4, tx=adamw(1.0, eps=10.0, weight_decay=0.0))
        sb = synthetic_batch(cfg, 70)
        b = Batch(sb.inputs.to(DEV), sb.labels.to(DEV))
        before = {n: v.detach().double().cpu().clone() for n, v in tr.state.params.state_dict().items()}
        tr.step(b)
        torch.cuda.synchronize()
        tr.finalize()
        assert tr.pp_kernel is not None
        after = {n: v.detach().double().cpu() for n, v in tr.state.params.state_dict().items()}
    finally:
        os.environ.pop("JDT_PP_CHAIN", None)
    want = mlp_grads_fp64({n: v.float() for n, v in before.items()}, MLP(pp_mlp_dims(cfg, L)).names, sb.inputs,
                          sb.labels, n_mb=4)
    for n in want:
        d = before[n] - after[n]
        check_grad(10 * d / (1 - d.abs()), want[n], n)
