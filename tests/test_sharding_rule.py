"""T1: shard_params rule == the reference's (param_sharding.py:58-125), table in SURVEY §2.7."""
import logging

import pytest
import torch

from jax_distributed_tuts_amd.models.mlp import Classifier
from jax_distributed_tuts_amd.parallel.fsdp import Partitioned, shard_rule

SHAPES = {"input_dense/kernel": (784, 512), "input_dense/bias": (512,), "output_dense/kernel": (512, 10),
          "output_dense/bias": (10,)}


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_table_min16(n):
    want = {"input_dense/kernel": 0, "input_dense/bias": 0, "output_dense/kernel": 0, "output_dense/bias": None}
    for name, shape in SHAPES.items():
        d, names = shard_rule(shape, (None,) * len(shape), "data", n, 2 ** 4, name)
        assert d == want[name], name
        if d is not None:
            assert names[d] == "data"


@pytest.mark.parametrize("n", [2, 4, 8])
def test_table_default_min(n):
    for name, shape in SHAPES.items():
        d, _ = shard_rule(shape, (None,) * len(shape), "data", n, 2 ** 18, name)
        assert d == (0 if name == "input_dense/kernel" else None)


def test_local_shapes_n8():
    from jax_distributed_tuts_amd.parallel.fsdp import ShardedFlatParams

    class FakeMesh:
        def axis_size(self, a):
            return 8

        def axis_index(self, a):
            return 3

    sp = ShardedFlatParams(Classifier().param_specs(), FakeMesh(), "data", 16, "cpu")
    shp = {n: sp.local.offsets[n][1] for n in sp.local.names()}
    assert shp == {"input_dense/kernel": (98, 512), "input_dense/bias": (64,), "output_dense/kernel": (64, 10),
                   "output_dense/bias": (10,)}
    assert sp.global_num_params() == 407050


def test_rule_edge_cases(caplog):
    caplog.set_level(logging.INFO, logger="jdt.fsdp")
    d, names = shard_rule((64, 8), ("data", None), "data", 4, 0, "already")
    assert d is None and "already sharded" in caplog.text
    d, _ = shard_rule((7, 9), (None, None), "data", 4, 0, "odd")
    assert d is None and "Could not shard" in caplog.text
    d, _ = shard_rule((4,), (None,), "data", 2, 16, "tiny")
    assert d is None and "too small" in caplog.text
    # descending size order, skipping dims already named (B5 path: pre-partitioned input)
    d, names = shard_rule((12, 64), (None, "pipe"), "data", 4, 0, "pp")
    assert d == 0 and names == ("data", "pipe")


def test_shard_params_values():
    from jax_distributed_tuts_amd.parallel.fsdp import shard_params

    class FakeMesh:
        def axis_size(self, a):
            return 4

        def axis_index(self, a):
            return 2

    w = torch.arange(16 * 3, dtype=torch.float32).view(16, 3)
    out = shard_params({"w": w, "b": torch.zeros(3)}, FakeMesh(), "data", min_weight_size=4)
    assert isinstance(out["w"], Partitioned) and torch.equal(out["w"].value, w[8:12])
    assert out["w"].names == ("data", None) and out["w"].global_shape == (16, 3)
    assert not isinstance(out["b"], Partitioned)
