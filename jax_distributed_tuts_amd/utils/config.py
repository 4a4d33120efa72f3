"""Attribute-access config dicts (the reference uses ml_collections.ConfigDict,
data_paral.py:38-72, param_sharding.py:31-55), plus the reference's literal
configs with its access bugs fixed."""
from __future__ import annotations

import copy
from typing import Any


class ConfigDict(dict):
    """dict with attribute access; nested dicts become ConfigDicts."""

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        for k, v in list(self.items()):
            if isinstance(v, dict) and not isinstance(v, ConfigDict):
                super().__setitem__(k, ConfigDict(v))

    def __getattr__(self, k: str) -> Any:
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k: str, v: Any):
        self[k] = ConfigDict(v) if isinstance(v, dict) and not isinstance(v, ConfigDict) else v

    def copy_and_resolve_references(self):
        return copy.deepcopy(self)


def dp_config() -> ConfigDict:
    """data_paral.py:38-72 (values verbatim)."""
    data = ConfigDict(batch_size=128, num_classes=10, input_size=784)
    model = ConfigDict(hidden_size=512, dropout_rate=0.1, dtype="bfloat16", num_classes=data.num_classes,
                       data_axis_name="data", input_size=data.input_size, num_layers=2, act="silu")
    optimizer = ConfigDict(learning_rate=1e-3, num_minibatches=4)
    return ConfigDict(model=model, optimizer=optimizer, data=data, data_axis_name=model.data_axis_name, seed=69)


def fsdp_config() -> ConfigDict:
    """param_sharding.py:31-55 + the min_weight_size override at :244-246."""
    data = ConfigDict(batch_size=128, num_classes=10, input_size=784)
    model = ConfigDict(hidden_size=512, dropout_rate=0.1, dtype="bfloat16", num_classes=data.num_classes,
                       data_axis_name="data", lr=1e-4, input_size=data.input_size, num_layers=2, act="silu",
                       min_weight_size=2 ** 4)
    return ConfigDict(model=model, data=data, seed=6969, num_minibatches=4)
