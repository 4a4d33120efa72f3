"""Drop-in ``util.py`` API of the reference (util.py:1-185), MI355X-native.

Same names and signatures: ``print_exception``, ``Pytree``, ``Metrics``, ``Parameter``,
``TrainState``, ``Batch``, ``sim_multiCPU_dev``, ``accum_grads_loop``,
``accum_grads_scan``, ``accum_grads``, ``print_metrics``, ``get_num_params``.
Implementations live in ``jax_distributed_tuts_amd.utils``.
"""
from __future__ import annotations

import os

from jax_distributed_tuts_amd.utils.metrics import Metrics, print_exception, print_metrics  # noqa: F401
from jax_distributed_tuts_amd.utils.train_state import (  # noqa: F401
    AdamW,
    Batch,
    GradBuffer,
    Parameter,
    Pytree,
    SGD,
    TrainState,
    accum_grads,
    accum_grads_loop,
    accum_grads_scan,
    adamw,
    get_num_params,
    sgd,
)
from jax_distributed_tuts_amd.utils.rng import PRNGKey, fold_rng_over_axis, split  # noqa: F401
from jax_distributed_tuts_amd.ops.autograd import softmax_cross_entropy_with_integer_labels  # noqa: F401


def sim_multiCPU_dev(device_count: int = 8):
    """util.py:31-38: simulate ``device_count`` devices without GPUs.

    The reference sets ``--xla_force_host_platform_device_count`` and hides CUDA
    (and forgets ``import os``).  Here it requests a gloo world of
    ``device_count`` CPU processes: entry points call
    ``jax_distributed_tuts_amd.runtime.launch.run``, which spawns them."""
    os.environ["JDT_SIM_CPU"] = str(int(device_count))
    os.environ["HIP_VISIBLE_DEVICES"] = ""
    os.environ["CUDA_VISIBLE_DEVICES"] = ""
