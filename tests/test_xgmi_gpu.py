"""xGMI P2P collectives (comm/xgmi.py + comm/csrc/xgmi.hip) on the GPU box.

The box has one MI355X, so 2 and 4 processes share it: that drives the real
IPC export/open, the cross-process per-block barriers, both buffer parities
and graph capture; the cross-GPU link behaviour itself is exercised by the
self-test each communicator runs at construction on the 8-GPU node."""
import os

import pytest
import torch

from jax_distributed_tuts_amd.runtime.launch import spawn

from . import xgmi_workers as XW

pytestmark = pytest.mark.gpu


def _load(d, name, ws):
    return [torch.load(os.path.join(d, f"{name}_r{r}.pt"), weights_only=True) for r in range(ws)]


@pytest.mark.parametrize("ws", [2, 4])
def test_xgmi_collectives(tmp_path, ws):
    spawn(XW.collectives, ws, str(tmp_path), gpu=True)
    for r, o in enumerate(_load(tmp_path, "xg", ws)):
        assert o["ok"], f"rank {r}: communicator self-test failed"
        assert all(o["ar"].values()), o["ar"]
        assert o["fused"] and o["rs"] and o["ag"] and o["graph"], o
        assert o["err"] == 0


def test_dp_over_xgmi_matches_single_device(tmp_path):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    spawn(XW.dp_xgmi, 2, str(tmp_path), gpu=True)
    res = _load(tmp_path, "dpx", 2)
    assert all(o["comm"] == "xgmi" for o in res)
    assert all(o["step"] == 8 for o in res)
    torch.testing.assert_close(res[0]["master"], res[1]["master"], rtol=0, atol=0)  # replicated exactly
    torch.testing.assert_close(res[0]["metrics"], res[1]["metrics"], rtol=0, atol=0)
    # single device, whole batch, same steps
    dev = torch.device("cuda", 0)
    st = init_dp(Classifier(dropout_rate=0.0), adamw(1e-3), 69, dev, None)
    b = synthetic_batch(dp_config(), 70)
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    for _ in range(8):
        tr.step(b)
    torch.cuda.synchronize()
    tr.finalize()
    d = (st.params.master.cpu() - res[0]["master"]).abs()
    assert float(d.max()) <= 2 * 1e-3 * 8 + 1e-6
    assert float((d > 5e-5).float().mean()) < 2e-3
    m, ref = res[0]["metrics"], tr.metrics.cpu()
    assert abs(float(m[0]) - float(ref[0])) <= 1e-3 * abs(float(ref[0])) + 1e-3
    assert float(m[1]) == float(ref[1]) and float(m[3]) == float(ref[3])
    assert abs(float(m[2]) - float(ref[2])) <= 4


@pytest.mark.parametrize("fused", [True, False])
def test_fsdp_over_xgmi_matches_single_device(tmp_path, fused):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.config import fsdp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    spawn(XW.fsdp_xgmi, 2, str(tmp_path), fused, gpu=True)
    res = _load(tmp_path, "fsx", 2)
    assert all(o["comm"] == "xgmi" for o in res)
    assert set(res[0]["xg_names"]) == {"input_dense/kernel", "input_dense/bias", "output_dense/kernel"}
    dev = torch.device("cuda", 0)
    st = init_fsdp(Classifier(dropout_rate=0.0), adamw(1e-3), 69, dev, None, "data", 16)
    b = synthetic_batch(fsdp_config(), 70)
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    tr = FSDPTrainer(st, None, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=fused))
    for _ in range(3):
        tr.step(b)
    torch.cuda.synchronize()
    sp = st.extra["sharded"]
    for n, d in res[0]["dims"].items():
        got = res[0]["local"][n] if d is None else torch.cat([o["local"][n] for o in res], dim=d)
        if d is None:
            torch.testing.assert_close(res[0]["local"][n], res[1]["local"][n], rtol=0, atol=0)
        diff = (got - sp.local.p(n).cpu()).abs()
        assert float(diff.max()) <= 2 * 1e-3 * 3 + 1e-6, n
        assert float((diff > 5e-5).float().mean()) < 5e-3, n
    m, ref = res[0]["metrics"], tr.metrics.cpu()
    assert abs(float(m[0]) - float(ref[0])) <= 1e-3 * abs(float(ref[0])) + 1e-3
    assert float(m[1]) == float(ref[1])
