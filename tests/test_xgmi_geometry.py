"""Host-side launch geometry of the xGMI collectives (comm/xgmi.py mirrors
``xg_geometry`` / the launch checks of comm/csrc/xgmi.hip).  The transport
calibration must time the trainer's own bucket, so every size a trainer sizes
its communicator for has to pass the two-shot launch check on that context."""
import pytest

from jax_distributed_tuts_amd.comm.xgmi import XG_MAX_BLOCKS, allreduce_fits, geometry, part_len


def create_cap(cap_floats: int, world: int) -> int:
    """``jdt_xgmi_create``'s capacity (floats per buffer half) for a requested size."""
    return (cap_floats + 4 * XG_MAX_BLOCKS * world + 63) // 64 * 64


@pytest.mark.parametrize("world", range(2, 9))
@pytest.mark.parametrize("n", [1, 4, 1000, 4_099, 300_001, 407_054, 1_628_160, 13_000_001])
def test_trainer_bucket_fits_its_own_context(world, n):
    f = allreduce_fits(n, world, create_cap(n, world))
    assert f["twoshot"] and f["oneshot"]


@pytest.mark.parametrize("s", [4, 100, 1024, 1028, 50_884, 101_764, 2_000_000])
def test_geometry_covers_the_part(s):
    g, chunk = geometry(s)
    assert 8 <= g <= XG_MAX_BLOCKS and chunk % 4 == 0
    assert g * chunk >= s and (g - 1) * chunk < s + 4 * g


def test_too_small_context_is_rejected():
    n, world = 407_054, 8
    assert not allreduce_fits(n, world, n // 2)["twoshot"]
    assert allreduce_fits(n, world, part_len(n, world) * world + 4 * XG_MAX_BLOCKS * world)["twoshot"]
