"""CPU mirror of the run-ahead tile map (csrc/common.h ``xcd_column_tile``).

The run-ahead backward kernels derive each workgroup's (hidden block, input
chunk) tile from the XCD it runs on (HW_REG_XCC_ID) and its linear id L:
t = xcc * (G / 8) + L / 8.  Workgroups are dealt round-robin over the 8 XCDs
with an offset carried over from earlier dispatches, so the map must be a
bijection for EVERY offset, and all chunks of a hidden block must land on one
XCD (their partial sums meet in that XCD's L2).  The kernels also check the
bijection at run time with per-tile launch counters (GPU tests)."""
import pytest


def column_tile(L: int, xcc: int, gx: int, gy: int):
    G = gx * gy
    t = (xcc & 7) * (G // 8) + L // 8
    return t // gy, t % gy   # (hidden block bx, input chunk by)


@pytest.mark.parametrize("gx,gy", [(32, 7), (64, 7), (16, 7)])
@pytest.mark.parametrize("offset", range(8))
def test_column_tile_map_is_a_bijection_for_any_dispatch_offset(gx, gy, offset):
    G = gx * gy
    assert G % 8 == 0 and (G // 8) % gy == 0   # the kernels' launch condition (H % 128 == 0)
    seen = {}
    for L in range(G):
        xcc = (L + offset) % 8               # round-robin dealing with a carried-over offset
        bx, by = column_tile(L, xcc, gx, gy)
        assert 0 <= bx < gx and 0 <= by < gy
        assert (bx, by) not in seen, "two workgroups on one tile"
        seen[(bx, by)] = xcc
    assert len(seen) == G
    for bx in range(gx):                     # a hidden block's chunks share one XCD (one L2)
        assert len({seen[(bx, by)] for by in range(gy)}) == 1
    # neighbouring hidden blocks share the XCD too: 4 (= G / 8 / gy) whole blocks per XCD
    per = (G // 8) // gy
    for bx in range(0, gx, per):
        assert len({seen[(b, 0)] for b in range(bx, bx + per)}) == 1


def test_tile_to_xcd_assignment_is_stable_across_launches():
    """Why the map reads the real XCD: with the assumed XCD = L % 8, a tile's workgroup
    runs on XCD (L + offset) % 8, and the offset differs from launch to launch (it
    carries over from earlier dispatches), so the same tile -- and its L2-resident
    barrier / tile counters -- would move between L2s across launches.  Deriving the
    tile from the XCD it runs on pins every tile (and counter line) to one XCD."""
    gx, gy, G = 32, 7, 224
    assumed = [{column_tile(L, L % 8, gx, gy): (L + off) % 8 for L in range(G)} for off in (0, 1)]
    assert any(assumed[0][t] != assumed[1][t] for t in assumed[0])      # moves between launches
    actual = [{column_tile(L, (L + off) % 8, gx, gy): (L + off) % 8 for L in range(G)} for off in (0, 1, 5)]
    assert all(actual[0][t] == a[t] for a in actual[1:] for t in actual[0])   # pinned
