"""Host-side checks of the one-launch N > 1 step's exchange geometry
(comm/tile_exchange.py, ops/csrc/common.h tx_tile and its callers in mlp_fused.hip /
mlp_deep.hip): every payload position a workgroup's threads move lies inside
TILE_PAYLOAD, no two threads of a workgroup share a position, and the tile counts match
the backward kernels' grids.  Pure index arithmetic mirrored from the kernels."""
import pytest

from jax_distributed_tuts_amd.comm.tile_exchange import SELFTEST_TILES, TILE_PAYLOAD
from jax_distributed_tuts_amd.parallel.fused_mlp import FusedMLPDeep

NT, NW, C = 512, 8, 10


def positions(ntile: int, chunk0: bool, lead: bool, top: bool = True):
    """{thread: [payload offsets]} as the kernels assign them (float4 slots expanded)."""
    out = {}
    for tid in range(NT):
        w, lane = tid >> 6, tid & 63
        p = []
        if w < ntile:
            p += [w * 256 + lane * 4 + e for e in range(4)]
            if lead and tid < 4:
                p.append(9 * 256 + 64 + tid)           # metric slot
        elif chunk0 and w == NW - 1:
            p += [7 * 256 + lane * 4 + e for e in range(4)]   # db (deep) / dW2 (2-layer)
            if top:
                p += [8 * 256 + lane * 4 + e for e in range(4)]
            if lead and lane < C:
                p.append(9 * 256 + lane)               # head / output bias
        out[tid] = p
    return out


@pytest.mark.parametrize("ntile,top", [(7, True), (7, False), (4, True), (4, False)])
def test_payload_positions_fit_and_are_disjoint(ntile, top):
    for chunk0, lead in ((False, False), (True, False), (True, True)):
        pos = positions(ntile, chunk0, lead, top)
        flat = [x for v in pos.values() for x in v]
        assert max(flat) < TILE_PAYLOAD and min(flat) >= 0
        assert len(flat) == len(set(flat)), (ntile, chunk0, lead)
    assert TILE_PAYLOAD % 4 == 0


def test_tile_counts_match_the_grids():
    # mlp2_bwd / md_bwd layer 0: (512 / 16) column blocks x (784 / 112) input chunks;
    # md_bwd layers >= 1: (512 / 16) x (512 / 64)
    assert FusedMLPDeep.tx_tiles(1) == 32 * 7
    assert FusedMLPDeep.tx_tiles(3) == 32 * 7 + 2 * 32 * 8
    eng = FusedMLPDeep.__new__(FusedMLPDeep)
    bases = [eng.tx_base(i) for i in range(3)]
    assert bases == [0, 224, 480]
    assert SELFTEST_TILES <= 32 * 7


@pytest.mark.parametrize("W", [2, 4, 8])
def test_fsdp_ownership_covers_every_element_once(W):
    """The FSDP one-launch exchange (mlp_fused.hip mlp2_bwd FX): for every tile, the owner
    set the kernel waits on (owner_of) contains every element's owner, every owner's local
    state index lies inside its shard, and over all tiles each W1 / W2 / b1 element is
    updated by exactly one rank -- the reference's dim-0 shards."""
    H, KC, NCH, NB = 512, 112, 7, 32
    rpq, hpq = 784 // W, H // W
    seen_w1 = [[0] * H for _ in range(784)]
    seen_h = [0] * H
    for bx in range(NB):
        j0 = bx * 16
        for by in range(NCH):
            T = bx * NCH + by
            kc0 = by * KC
            o_lo, o_hi, ob, orep = kc0 // rpq, (kc0 + KC - 1) // rpq, j0 // hpq, T % W
            # the kernel's partial stores reach o_lo and o_hi only: no middle owner
            assert o_hi - o_lo <= 1
            owners = {q for q in range(W) if o_lo <= q <= o_hi or (by == 0 and q == ob) or q == orep}
            for r in range(kc0, kc0 + KC):
                o = r // rpq
                assert o in owners and 0 <= r - o * rpq < rpq
                for c in range(j0, j0 + 16):
                    seen_w1[r][c] += 1
            if by == 0:
                for n in range(16):
                    assert ob in owners and 0 <= j0 + n - ob * hpq < hpq
                    seen_h[j0 + n] += 1
            assert orep in owners
    assert all(v == 1 for row in seen_w1 for v in row)
    assert all(v == 1 for v in seen_h)


def test_fx_owner_span_guards_the_allowed_worlds():
    """fsdp._tile_exchange admits W only when each 112-row chunk has <= 2 owners:
    true for W = 2 / 4 / 8, false for W = 16 (49-row shards) and non-divisors."""
    from jax_distributed_tuts_amd.comm.tile_exchange import fx_owner_span

    assert [fx_owner_span(W) for W in (1, 2, 4, 8)] == [1, 2, 2, 2]
    assert fx_owner_span(16) > 2 and fx_owner_span(3) > 2
