"""--deterministic (JDT_DETERMINISTIC=1): two identical runs give bitwise-identical
parameters and metrics.  The fused engines then sum per-column-
block partial logits in block order instead of with fp32 atomics -- the 2-layer DP run
is the headline path (run-ahead steps, persistent multi-step launch)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _dp_run(num_layers, steps=6):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    st = init_dp(Classifier(num_layers=num_layers), adamw(1e-3), 69, DEV)
    b = synthetic_batch(dp_config(), 70)
    b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    for _ in range(2):
        tr.step(b)
    tr.capture(b, steps_per_graph=2)
    tr.run_steps(b, steps - 2)
    tr.finalize()
    torch.cuda.synchronize()
    assert tr.fused is not None and tr.fused.det_logits is not None
    if num_layers == 2:
        # the headline kernel: run-ahead steps, a 2-step replay as ONE persistent launch
        assert tr.fused.ahead_ok and tr.fused.pst_ok and tr.multi is not None
    return st.params.master.cpu().clone(), tr.metrics.cpu().clone()


def _pp_run(steps=4):
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch

    cfg = dp_config()
    tr = build_mlp_pipeline(cfg, Mesh({"data": 1, "pipe": 1}), DEV, n_hidden_layers=4, num_microbatches=4)
    b = synthetic_batch(cfg, 70)
    b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
    for _ in range(steps):
        tr.step(b)
    tr.finalize()
    torch.cuda.synchronize()
    assert tr.deep_engine is not None and tr.deep_engine.det_logits is not None
    return tr.state.params.master.cpu().clone(), tr.metrics.cpu().clone()


@pytest.mark.parametrize("run", ["dp2", "dp4", "pp"])
def test_deterministic_runs_are_bitwise_identical(monkeypatch, run):
    monkeypatch.setenv("JDT_DETERMINISTIC", "1")
    fn = {"dp2": lambda: _dp_run(2), "dp4": lambda: _dp_run(4), "pp": _pp_run}[run]
    (p1, m1), (p2, m2) = fn(), fn()
    assert torch.equal(p1, p2), float((p1 - p2).abs().max())
    assert torch.equal(m1, m2)
