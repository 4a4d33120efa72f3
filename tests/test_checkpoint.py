"""Checkpoint layout validation and trainer invalidation."""
import json
import os

import pytest
import torch

from jax_distributed_tuts_amd.models.mlp import Classifier
from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
from jax_distributed_tuts_amd.utils import checkpoint
from jax_distributed_tuts_amd.utils.train_state import adamw


def _dp(num_layers=2):
    st = init_dp(Classifier(num_layers=num_layers), adamw(1e-3), 69, "cpu")
    return st, DataParallelTrainer(st, None, DPConfig(4, "fused"))


def _batch():
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.utils.config import dp_config

    return synthetic_batch(dp_config(), 70)


def test_roundtrip_and_invalidate(tmp_path):
    st, tr = _dp()
    b = _batch()
    tr.step(b)
    checkpoint.save(st, str(tmp_path), tr.metrics)
    ref = {k: v.clone() for k, v in st.params.state_dict().items()}
    tr.step(b)
    tr.graph = "stale-graph-sentinel"
    checkpoint.restore(st, str(tmp_path), tr.metrics)
    assert tr.graph is None  # derived device state dropped
    for k, v in st.params.state_dict().items():
        torch.testing.assert_close(v, ref[k], rtol=0, atol=0)
    assert st.step == 1 and int(st.opt_state["count"]) == 1


def test_restore_rejects_other_model(tmp_path):
    st, tr = _dp(2)
    checkpoint.save(st, str(tmp_path))
    st4, _ = _dp(4)
    with pytest.raises(ValueError):
        checkpoint.restore(st4, str(tmp_path))


def test_restore_rejects_same_size_other_layout(tmp_path):
    """Same total size, different views: rejected on the view table, not numel."""
    st, _ = _dp(2)
    checkpoint.save(st, str(tmp_path))
    man_f = os.path.join(str(tmp_path), "rank0.json")
    man = json.load(open(man_f))
    man["views"]["input_dense/kernel"]["shape"] = [512, 784]
    json.dump(man, open(man_f, "w"))
    with pytest.raises(ValueError, match="shape"):
        checkpoint.restore(st, str(tmp_path))


def test_restore_rejects_other_world_size(tmp_path):
    st, _ = _dp(2)
    checkpoint.save(st, str(tmp_path))
    man_f = os.path.join(str(tmp_path), "rank0.json")
    man = json.load(open(man_f))
    man["world_size"] = 8
    json.dump(man, open(man_f, "w"))
    with pytest.raises(ValueError, match="8-rank"):
        checkpoint.restore(st, str(tmp_path))


def test_restore_rejects_other_optimizer_before_touching_state(tmp_path):
    """An AdamW checkpoint restored into an SGD state (or back) is refused with a
    ValueError naming the optimizer slots, and the live params are left untouched."""
    from jax_distributed_tuts_amd.utils.train_state import sgd

    st, tr = _dp()
    tr.step(_batch())
    checkpoint.save(st, str(tmp_path))
    st2 = init_dp(Classifier(), sgd(0.1), 7, "cpu")
    before = st2.params.master.clone()
    with pytest.raises(ValueError, match="optimizer state"):
        checkpoint.restore(st2, str(tmp_path))
    torch.testing.assert_close(st2.params.master, before, rtol=0, atol=0)


def test_free_port_with_low_ephemeral_range(monkeypatch):
    """An ephemeral range starting at 1024 leaves no room below it: bind(0) fallback."""
    import builtins
    import io

    from jax_distributed_tuts_amd.runtime import launch

    real_open = builtins.open

    def fake_open(path, *a, **k):
        if str(path) == "/proc/sys/net/ipv4/ip_local_port_range":
            return io.StringIO("1024\t65535\n")
        return real_open(path, *a, **k)

    monkeypatch.setattr(builtins, "open", fake_open)
    port = launch.free_port()
    assert 0 < port < 65536
