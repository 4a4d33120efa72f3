"""``Mesh(unit_groups=True)``: a 1-member axis with a real process group, so a
one-device job runs the N > 1 collective schedule (used on the GPU box to put RCCL
calls inside captured step graphs, tests/test_rccl_capture_gpu.py)."""
import os

import torch

from jax_distributed_tuts_amd.runtime.launch import spawn

from . import dist_workers as W


def test_unit_group_schedule_trains_like_one_device(tmp_path):
    spawn(W.unit_groups, 1, str(tmp_path))
    o = torch.load(os.path.join(tmp_path, "unit_r0.pt"), weights_only=True)
    assert not o["active_False"] and o["active_True"]
    assert not o["dp_coll_False"] and o["dp_coll_True"]
    assert o["fsdp_n1_False"] and not o["fsdp_n1_True"]
    torch.testing.assert_close(o["dp_True"], o["dp_False"], rtol=0, atol=0)
    torch.testing.assert_close(o["fsdp_True"], o["fsdp_False"], rtol=1e-6, atol=1e-7)
