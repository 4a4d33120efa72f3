"""Host-side checks of the in-kernel GPipe stage step (parallel/pp_kernel.py,
ops/csrc/pp_stage.hip): which pipeline splits it takes (one 512-wide layer per stage,
784 inputs on stage 0, the head on the last -- BASELINE config #4's 8-stage MLP), the
inbox slot size, and the ctypes mirror of the kernel's argument struct."""
import ctypes

import pytest

from jax_distributed_tuts_amd.parallel import pp_kernel as PK
from jax_distributed_tuts_amd.parallel.pipeline import mlp_stage
from pipeline_parallel import pp_mlp_dims
from jax_distributed_tuts_amd.utils.config import dp_config


@pytest.mark.parametrize("S,n_hidden,fits", [(8, 8, True), (4, 4, True), (2, 2, True), (8, 7, False),
                                             (4, 3, False), (2, 3, False)])
def test_stage_kernel_takes_one_layer_per_stage(S, n_hidden, fits):
    dims = pp_mlp_dims(dp_config(), n_hidden)
    got = [PK.stage_fits(mlp_stage(dims, S, s), s == 0, s == S - 1) for s in range(S)]
    assert all(got) == fits, got
    if fits:
        # stage 0 takes the data, the last carries the head, the rest one hidden layer each
        assert mlp_stage(dims, S, 0).dims == [784, 512]
        assert mlp_stage(dims, S, S - 1).dims == [512, 512, 10]
        assert [mlp_stage(dims, S, s).layer_id_base for s in range(S)] == list(range(S))


def test_slot_holds_activation_and_its_transpose():
    # H [mb][512] + H^T [512][mbp] bf16, mbp = mb rounded up to the 32-deep dW k-steps
    assert PK.slot_bytes(64) == 64 * 512 * 2 + 512 * 64 * 2
    assert PK.slot_bytes(32) == 32 * 512 * 2 + 512 * 32 * 2


def test_args_mirror_is_packed_like_the_kernel_struct():
    from jax_distributed_tuts_amd.ops import _lib

    assert _lib.lib().jdt_pp_stage_args_size() == ctypes.sizeof(PK.PsArgs)
