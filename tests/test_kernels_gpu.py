"""T4: every HIP kernel vs the fp32 torch reference of the same op (CPU path of
ops/kernels.py, which rounds matmul operands to bf16 like the kernels do)."""
import pytest
import torch

from jax_distributed_tuts_amd.ops import kernels as kern

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= atol + rtol * scale, f"max err {err} (scale {scale})"


def _mk(shape, dtype, layout_t=False, seed=0):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(*shape, generator=g)
    return t.to(dtype)


@pytest.fixture(params=["dma", "preload", "pipelined"])
def gemm_path(request):
    """Run a GEMM test through the LDS-DMA kernel (bf16 operands, tile-aligned
    shapes), the all-K-tiles-preloaded register kernel and the pipelined one."""
    from jax_distributed_tuts_amd.ops import _lib

    L = _lib.lib()
    L.jdt_gemm_set_dma(int(request.param == "dma"))
    L.jdt_gemm_set_preload(int(request.param != "pipelined"))
    yield request.param
    L.jdt_gemm_set_dma(1)
    L.jdt_gemm_set_preload(1)


@pytest.mark.parametrize("M,N,K", [(4, 512, 784), (16, 512, 784), (32, 10, 512), (128, 512, 784), (37, 70, 50),
                                   (256, 384, 256), (512, 512, 512), (64, 128, 2048), (96, 192, 128),
                                   (512, 1536, 512)])
@pytest.mark.parametrize("a_layout,b_layout", [("mk", "kn"), ("mk", "nk"), ("km", "kn"), ("km", "nk")])
@pytest.mark.parametrize("adt", [torch.bfloat16, torch.float32])
def test_gemm_layouts(M, N, K, a_layout, b_layout, adt, gemm_path):
    a = _mk((M, K) if a_layout == "mk" else (K, M), adt, seed=1)
    b = _mk((K, N) if b_layout == "kn" else (N, K), torch.bfloat16, seed=2)
    ref = kern.gemm(a, b, a_layout=a_layout, b_layout=b_layout, out_dtype=torch.float32)
    out = kern.gemm(a.to(DEV), b.to(DEV), a_layout=a_layout, b_layout=b_layout, out_dtype=torch.float32)
    _close(out, ref, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("act", ["none", "silu", "gelu", "relu"])
def test_gemm_fwd_epilogue(act):
    M, N, K_ = 64, 512, 784
    x = _mk((M, K_), torch.float32, seed=3)
    w = (_mk((K_, N), torch.float32, seed=4) * 0.05).to(torch.bfloat16)
    b = _mk((N,), torch.bfloat16, seed=5)
    zr = torch.empty(M, N, dtype=torch.bfloat16)
    ref = kern.gemm(x, w, bias=b, act=act, z_out=zr, keep_prob=0.9, seed=7, offset=11)
    zg = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    out = kern.gemm(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=act, z_out=zg, keep_prob=0.9, seed=7, offset=11)
    _close(zg, zr)
    _close(out, ref)
    # identical dropout mask (Philox bit parity CPU <-> GPU): where z > 0.5 every
    # activation is clearly nonzero, so a zero output can only be a dropped element
    sel = zr.float() > 0.5
    assert torch.equal((out.cpu() == 0)[sel], (ref == 0)[sel])
    assert 0.05 < float((ref == 0)[sel].float().mean()) < 0.15


def test_gemm_bwd_epilogue_and_dbias():
    M, N, K_ = 32, 512, 10
    dz = _mk((M, K_), torch.bfloat16, seed=6)
    w = _mk((N, K_), torch.bfloat16, seed=7)  # [in=N, out=K] kernel read "nk"
    z = _mk((M, N), torch.bfloat16, seed=8)
    db_r = torch.zeros(N)
    ref = kern.gemm(dz, w, b_layout="nk", z_in=z, act_bwd="silu", keep_prob=0.9, seed=3, offset=5, dbias=db_r)
    db_g = torch.zeros(N, device=DEV)
    out = kern.gemm(dz.to(DEV), w.to(DEV), b_layout="nk", z_in=z.to(DEV), act_bwd="silu", keep_prob=0.9, seed=3,
                 offset=5, dbias=db_g)
    _close(out, ref)
    _close(db_g, db_r, rtol=2e-2, atol=5e-2)


def test_gemm_accumulate_fp32():
    x = _mk((784, 32), torch.float32, seed=9)   # "km": x stored [M_rows=32?]
    dz = _mk((32, 512), torch.bfloat16, seed=10)
    x = _mk((32, 784), torch.float32, seed=9)
    acc_r = torch.ones(784, 512)
    kern.gemm(x, dz, a_layout="km", b_layout="kn", out=acc_r, accumulate=True)
    acc_g = torch.ones(784, 512, device=DEV)
    kern.gemm(x.to(DEV), dz.to(DEV), a_layout="km", b_layout="kn", out=acc_g, accumulate=True)
    _close(acc_g, acc_r, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("cfg", [-1, 14])
@pytest.mark.parametrize("a_layout,b_layout", [("mk", "kn"), ("mk", "nk"), ("km", "kn"), ("km", "nk")])
def test_gemm_dma_epilogues(a_layout, b_layout, cfg):
    """LDS-DMA kernel with every fused epilogue: bias + GELU + z_out + dropout +
    residual (forward), act' * mask + dbias (backward), fp32 accumulate, split-K.
    cfg 14: 128 x 128 tiles (64-wide transposed sub-images, LDS-staged epilogue)."""
    M, N, K_ = (128, 256, 512) if cfg < 0 else (256, 384, 512)
    a = _mk((M, K_) if a_layout == "mk" else (K_, M), torch.bfloat16, seed=61)
    b = (_mk((K_, N) if b_layout == "kn" else (N, K_), torch.float32, seed=62) * 0.05).to(torch.bfloat16)
    bias, res = _mk((N,), torch.bfloat16, seed=63), _mk((M, N), torch.bfloat16, seed=64)
    zr = torch.empty(M, N, dtype=torch.bfloat16)
    ref = kern.gemm(a, b, a_layout=a_layout, b_layout=b_layout, bias=bias, act="gelu", z_out=zr, keep_prob=0.9,
                    seed=7, offset=11, resid=res)
    zg = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    out = kern.gemm(a.to(DEV), b.to(DEV), a_layout=a_layout, b_layout=b_layout, bias=bias.to(DEV), act="gelu",
                    z_out=zg, keep_prob=0.9, seed=7, offset=11, resid=res.to(DEV), cfg=cfg)
    _close(zg, zr)
    _close(out, ref)
    z = _mk((M, N), torch.bfloat16, seed=65)
    db_r, db_g = torch.zeros(N), torch.zeros(N, device=DEV)
    ref = kern.gemm(a, b, a_layout=a_layout, b_layout=b_layout, z_in=z, act_bwd="silu", keep_prob=0.9, seed=3,
                    offset=5, dbias=db_r)
    out = kern.gemm(a.to(DEV), b.to(DEV), a_layout=a_layout, b_layout=b_layout, z_in=z.to(DEV), act_bwd="silu",
                    keep_prob=0.9, seed=3, offset=5, dbias=db_g, cfg=cfg)
    _close(out, ref)
    _close(db_g, db_r, rtol=2e-2, atol=5e-2)
    for splits in (-1, 4, 8):
        acc_r = torch.full((M, N), 0.5)
        kern.gemm(a, b, a_layout=a_layout, b_layout=b_layout, out=acc_r, accumulate=True)
        acc_g = torch.full((M, N), 0.5, device=DEV)
        kern.gemm(a.to(DEV), b.to(DEV), a_layout=a_layout, b_layout=b_layout, out=acc_g, accumulate=True,
                  cfg=11 if cfg < 0 else cfg, splits=splits)
        _close(acc_g, acc_r, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("cfg,r", [(10, 1), (10, 2), (11, 1), (11, 2), (12, 1), (13, 4), (14, 1)])
@pytest.mark.parametrize("a_layout,b_layout", [("mk", "kn"), ("km", "nk")])
def test_gemm_vec_epilogue_bit_identical(cfg, r, a_layout, b_layout):
    """The vectorised LDS-image epilogue (gemm_finish_vec) computes every element
    with the same arithmetic as the per-element one: outputs bit-identical for the
    forward epilogue (bias, GELU, z_out, dropout, residual), the backward one (act'
    * mask, dbias), bf16 / fp32 accumulate and split-K; at each tile config and
    K sub-tiles per ring slot (r)."""
    from jax_distributed_tuts_amd.ops import _lib

    L = _lib.lib()
    M, N, K_ = 256, 384, 512
    a = _mk((M, K_) if a_layout == "mk" else (K_, M), torch.bfloat16, seed=81).to(DEV)
    b = (_mk((K_, N) if b_layout == "kn" else (N, K_), torch.float32, seed=82) * 0.05).to(torch.bfloat16).to(DEV)
    bias, res = _mk((N,), torch.bfloat16, seed=83).to(DEV), _mk((M, N), torch.bfloat16, seed=84).to(DEV)
    z = _mk((M, N), torch.bfloat16, seed=85).to(DEV)
    kw = dict(a_layout=a_layout, b_layout=b_layout, cfg=cfg)

    def run():
        zo = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        f = kern.gemm(a, b, bias=bias, act="gelu", z_out=zo, keep_prob=0.9, seed=7, offset=11, resid=res, **kw)
        db = torch.zeros(N, device=DEV)
        g = kern.gemm(a, b, z_in=z, act_bwd="silu", keep_prob=0.9, seed=3, offset=5, dbias=db, **kw)
        acc16 = res.clone()
        kern.gemm(a, b, out=acc16, accumulate=True, **kw)
        acc32 = [torch.full((M, N), 0.5, device=DEV) for _ in range(2)]
        kern.gemm(a, b, out=acc32[0], accumulate=True, **kw)
        kern.gemm(a, b, out=acc32[1], accumulate=True, splits=4, **kw)
        torch.cuda.synchronize()
        return [zo, f, g, acc16, acc32[0], acc32[1]], db

    L.jdt_gemm_set_r(r)
    try:
        outs_v, db_v = run()
        L.jdt_gemm_set_epi_vec(0)
        outs_e, db_e = run()
    finally:
        L.jdt_gemm_set_epi_vec(1)
        L.jdt_gemm_set_r(-1)
    for x, y in zip(outs_v, outs_e):
        assert torch.equal(x, y)
    _close(db_v, db_e, rtol=1e-5, atol=1e-4)  # fp32 atomics: summation order differs


@pytest.mark.parametrize("cfg", [20, 21, 22, 23, 24, 25, 26, 27])
@pytest.mark.parametrize("a_layout,b_layout", [("mk", "kn"), ("mk", "nk"), ("km", "kn"), ("km", "nk")])
def test_gemm_mfma32_tiles(cfg, a_layout, b_layout):
    """32x32x16-MFMA LDS-DMA tiles (64 x 64 .. 128 x 128, 3- and 4-slot rings, 4 and 8
    waves; transposed operands through the 32-column tr-read fragment): every fused
    epilogue and split-K against the 16x16x32 128 x 128 tile (same arithmetic, a
    different in-MFMA summation order: bf16-rounding close, not bit-identical) and the
    fp32 product against torch."""
    M, N, K_ = 512, 512, 1024
    a = _mk((M, K_) if a_layout == "mk" else (K_, M), torch.bfloat16, seed=81).to(DEV)
    b = (_mk((K_, N) if b_layout == "kn" else (N, K_), torch.float32, seed=82) * 0.05).to(torch.bfloat16).to(DEV)
    bias, res = _mk((N,), torch.bfloat16, seed=83).to(DEV), _mk((M, N), torch.bfloat16, seed=84).to(DEV)
    z = _mk((M, N), torch.bfloat16, seed=85).to(DEV)

    def run(c):
        kw = dict(a_layout=a_layout, b_layout=b_layout, cfg=c)
        zo = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        f = kern.gemm(a, b, bias=bias, act="gelu", z_out=zo, resid=res, **kw)
        db = torch.zeros(N, device=DEV)
        g = kern.gemm(a, b, z_in=z, act_bwd="silu", dbias=db, **kw)
        acc32 = [torch.full((M, N), 0.5, device=DEV) for _ in range(2)]
        kern.gemm(a, b, out=acc32[0], accumulate=True, splits=1, **kw)
        kern.gemm(a, b, out=acc32[1], accumulate=True, splits=4, **kw)
        torch.cuda.synchronize()
        return [zo, f, g, acc32[0], acc32[1]], db

    outs, db = run(cfg)
    ref_outs, ref_db = run(14)
    for x, y in zip(outs, ref_outs):
        _close(x.float(), y.float(), rtol=2e-2, atol=2e-2)
    _close(db, ref_db, rtol=1e-3, atol=1e-2)
    A = a.float() if a_layout == "mk" else a.float().t()
    B = b.float() if b_layout == "kn" else b.float().t()
    for o in outs[3:]:
        _close(o - 0.5, A @ B, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("cfg", [15, 16, 17, 18])
@pytest.mark.parametrize("a_layout,b_layout", [("mk", "kn"), ("mk", "nk"), ("km", "kn"), ("km", "nk")])
def test_gemm_8wave_tiles_match_4wave(cfg, a_layout, b_layout):
    """8-wave LDS-DMA tiles (two waves per SIMD; 128 x 128, 256 x 128, 128 x 256)
    accumulate every output element in the same K order as the 4-wave 128 x 128
    tile: bit-identical outputs for the full forward / backward epilogues,
    bf16 / fp32 accumulate and split-K; and close to the fp32 reference."""
    M, N, K_ = 512, 512, 1024
    a = _mk((M, K_) if a_layout == "mk" else (K_, M), torch.bfloat16, seed=91).to(DEV)
    b = (_mk((K_, N) if b_layout == "kn" else (N, K_), torch.float32, seed=92) * 0.05).to(torch.bfloat16).to(DEV)
    bias, res = _mk((N,), torch.bfloat16, seed=93).to(DEV), _mk((M, N), torch.bfloat16, seed=94).to(DEV)
    z = _mk((M, N), torch.bfloat16, seed=95).to(DEV)

    def run(c):
        kw = dict(a_layout=a_layout, b_layout=b_layout, cfg=c)
        zo = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        f = kern.gemm(a, b, bias=bias, act="gelu", z_out=zo, keep_prob=0.9, seed=7, offset=11, resid=res, **kw)
        db = torch.zeros(N, device=DEV)
        g = kern.gemm(a, b, z_in=z, act_bwd="silu", keep_prob=0.9, seed=3, offset=5, dbias=db, **kw)
        acc16 = res.clone()
        kern.gemm(a, b, out=acc16, accumulate=True, **kw)
        acc32 = [torch.full((M, N), 0.5, device=DEV) for _ in range(2)]
        kern.gemm(a, b, out=acc32[0], accumulate=True, splits=1, **kw)
        kern.gemm(a, b, out=acc32[1], accumulate=True, splits=4, **kw)
        torch.cuda.synchronize()
        return [zo, f, g, acc16, acc32[0], acc32[1]], db

    outs, db = run(cfg)
    ref_outs, ref_db = run(14)
    for x, y in zip(outs, ref_outs):
        assert torch.equal(x, y)
    _close(db, ref_db, rtol=1e-5, atol=1e-4)  # fp32 atomics: summation order differs
    A = a.float() if a_layout == "mk" else a.float().t()
    B = b.float() if b_layout == "kn" else b.float().t()
    _close(outs[4] - 0.5, A @ B, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize("tile", [32, 64, 128])
def test_gemm_group_tiles(tile):
    """Grouped launch at each tile size (forced): a weight gradient (km x kn, fp32
    accumulate, split-K) next to an input gradient (mk x nk, act' + mask + dbias)."""
    from jax_distributed_tuts_amd.ops import _lib

    M, N, K_ = 256, 384, 1024
    h = _mk((K_, M), torch.bfloat16, seed=71)
    dz = _mk((K_, N), torch.bfloat16, seed=72)
    w = (_mk((M, N), torch.float32, seed=73) * 0.05).to(torch.bfloat16)
    zin = _mk((K_, M), torch.bfloat16, seed=74)
    dw_r, dw_g = torch.full((M, N), 0.25), torch.full((M, N), 0.25, device=DEV)
    db_r, db_g = torch.zeros(M), torch.zeros(M, device=DEV)
    kern.gemm(h, dz, a_layout="km", b_layout="kn", out=dw_r, accumulate=True)
    dx_r = kern.gemm(dz, w, a_layout="mk", b_layout="nk", z_in=zin, act_bwd="gelu", keep_prob=0.9, seed=5,
                     offset=9, dbias=db_r)
    _lib.lib().jdt_gemm_set_group_tile(tile)
    try:
        with kern.gemm_group():
            kern.gemm(h.to(DEV), dz.to(DEV), a_layout="km", b_layout="kn", out=dw_g, accumulate=True)
            dx_g = kern.gemm(dz.to(DEV), w.to(DEV), a_layout="mk", b_layout="nk", z_in=zin.to(DEV), act_bwd="gelu",
                             keep_prob=0.9, seed=5, offset=9, dbias=db_g)
        torch.cuda.synchronize()
    finally:
        _lib.lib().jdt_gemm_set_group_tile(0)
    _close(dw_g, dw_r, rtol=1e-3, atol=2e-3)
    _close(dx_g, dx_r)
    _close(db_g, db_r, rtol=2e-2, atol=5e-2)


def test_gemm_batched():
    for (m, k, n) in ((64, 96, 80), (64, 128, 64)):  # register-staged / LDS-DMA
        a = _mk((3, m, k), torch.bfloat16, seed=11)
        b = _mk((3, k, n), torch.bfloat16, seed=12)
        ref = kern.gemm(a, b, out_dtype=torch.float32)
        out = kern.gemm(a.to(DEV), b.to(DEV), out_dtype=torch.float32)
        _close(out, ref, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("M,C", [(4, 10), (128, 10), (33, 1000), (64, 2048), (37, 512), (1500, 768), (9, 1000 + 8)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_xent(M, C, dt):
    z = (_mk((M, C), torch.float32, seed=13) * 3).to(dt)
    y = torch.randint(0, C, (M,), generator=torch.Generator().manual_seed(1)).to(torch.int32)
    y[0] = -1  # ignored row
    d_r = torch.empty(M, C, dtype=torch.bfloat16)
    db_r, m_r, l_r = torch.zeros(C), torch.zeros(4), torch.zeros(M)
    kern.softmax_xent(z, y, grad_scale=1 / M, dlogits=d_r, dbias=db_r, metrics=m_r, row_loss=l_r)
    d_g = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    db_g, m_g, l_g = torch.zeros(C, device=DEV), torch.zeros(4, device=DEV), torch.zeros(M, device=DEV)
    kern.softmax_xent(z.to(DEV), y.to(DEV), grad_scale=1 / M, dlogits=d_g, dbias=db_g, metrics=m_g, row_loss=l_g)
    _close(l_g, l_r, rtol=1e-4, atol=1e-4)
    _close(d_g, d_r, rtol=1e-2, atol=1e-4)
    _close(db_g, db_r, rtol=1e-2, atol=1e-4)
    _close(m_g, m_r, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("M,C", [(2048, 2048), (512, 2048), (37, 512), (33, 1000)])
def test_xent_metric_slab_fold(M, C):
    """Per-workgroup metric rows (softmax_xent mslab) + the step-end fold (slab sums, slot,
    step advance) == the slot atomics + plain fold; the slab comes back zeroed.  (33, 1000)
    takes the narrow kernel, which keeps the atomics: the fold still adds the slot."""
    z = (_mk((M, C), torch.float32, seed=21) * 3).to(torch.bfloat16).to(DEV)
    y = torch.randint(0, C, (M,), generator=torch.Generator().manual_seed(2)).to(torch.int32).to(DEV)
    y[1] = -1
    runs = []
    for use_slab in (False, True):
        slot, run = torch.zeros(4, device=DEV), torch.full((4,), 2.0, device=DEV)
        slab = torch.zeros(1024, 4, device=DEV) if use_slab else None
        step = torch.zeros(1, dtype=torch.int32, device=DEV) if use_slab else None
        d = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
        for _ in range(2):
            # two CE launches per fold (the per-microbatch schedule): the rows accumulate
            for _ in range(2):
                kern.softmax_xent(z, y, grad_scale=1 / M, dlogits=d, metrics=slot, mslab=slab)
            kern.metrics_fold_(run, slot, slab=slab, step=step)
        torch.cuda.synchronize()
        runs.append(run.cpu())
        if use_slab:
            assert int(step.item()) == 2
            assert float(slab.abs().sum()) == 0.0 and float(slot.abs().sum()) == 0.0
    _close(runs[1], runs[0], rtol=1e-5, atol=1e-3)
    assert float(runs[1][1]) == 2.0 + 4 * (M - 1)


@pytest.mark.parametrize("n", [407050, 3_000_001])   # one partial round / several rounds of AW_U groups per thread
def test_adamw_and_step_counter(n):
    g = torch.Generator().manual_seed(0)
    p = torch.randn(n, generator=g)
    gr = torch.randn(n, generator=g)
    st = {}
    for dev in ("cpu", DEV):
        P, G = p.clone().to(dev), gr.clone().to(dev)
        m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
        step, ticket = torch.zeros(1, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int32, device=dev)
        for _ in range(3):
            G.copy_(gr.to(dev))
            kern.adamw_step(P, G, m, v, sh, lr=1e-3, grad_scale=0.25, step=step, ticket=ticket)
        st[dev] = (P.cpu(), sh.cpu(), step.cpu(), G.cpu())
    _close(st[DEV][0], st["cpu"][0], rtol=1e-5, atol=1e-6)
    assert int(st[DEV][2]) == 3 and float(st[DEV][3].abs().max()) == 0.0
    _close(st[DEV][1], st["cpu"][1], rtol=1e-2, atol=1e-2)


def test_act_bwd():
    M, N = 48, 300
    dh, z = _mk((M, N), torch.bfloat16, seed=1), _mk((M, N), torch.bfloat16, seed=2)
    step = torch.tensor([5], dtype=torch.int32)
    db_r = torch.zeros(N)
    r = kern.act_bwd(dh, z, "gelu", keep_prob=0.8, seed=9, offset=3, step=step, dbias=db_r)
    db_g = torch.zeros(N, device=DEV)
    o = kern.act_bwd(dh.to(DEV), z.to(DEV), "gelu", keep_prob=0.8, seed=9, offset=3, step=step.to(DEV), dbias=db_g)
    _close(o, r)
    _close(db_g, db_r, rtol=1e-2, atol=1e-2)


def test_dp_step_gpu_matches_cpu():
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(0)
    x = torch.randn(128, 784, generator=g)
    y = torch.randint(0, 10, (128,), generator=g).to(torch.int32)
    res = {}
    for dev in ("cpu", DEV):
        model = Classifier(dropout_rate=0.1)
        st = init_dp(model, adamw(1e-3), 69, dev)
        tr = DataParallelTrainer(st, None, DPConfig(4, "loop"))
        for _ in range(3):
            tr.step(Batch(x.to(dev), y.to(dev)))
        res[dev] = (st.params.master.cpu(), tr.metrics.cpu())
    _close(res[DEV][0], res["cpu"][0], rtol=1e-2, atol=2e-3)
    _close(res[DEV][1], res["cpu"][1], rtol=1e-2, atol=1e-2)


def test_dp_graph_replay_matches_eager():
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(0)
    x = torch.randn(128, 784, generator=g).to(DEV)
    y = torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV)
    out = []
    for use_graph in (False, True):
        st = init_dp(Classifier(), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, "loop"))
        tr.step(Batch(x, y))
        if use_graph:
            tr.capture(Batch(x, y))
        for _ in range(5):
            tr.step(Batch(x, y))
        torch.cuda.synchronize()
        out.append((st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item())))
    assert out[0][2] == out[1][2] == 6
    torch.testing.assert_close(out[1][0], out[0][0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(out[1][1], out[0][1], rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("splits", [1, 3, 7, 16])
@pytest.mark.parametrize("M,N,K_,cfg", [(32, 512, 784, 0), (128, 10, 512, 4), (784, 512, 128, 2)])
def test_gemm_split_k(splits, M, N, K_, cfg, gemm_path):
    """In-kernel split-K (slab + last-arriver combine) must match the single-slice result,
    including the fused epilogue (bias/act/dropout) and fp32 accumulate."""
    x = _mk((M, K_), torch.float32, seed=21)
    w = (_mk((K_, N), torch.float32, seed=22) * 0.05).to(torch.bfloat16)
    b = _mk((N,), torch.bfloat16, seed=23)
    ref = kern.gemm(x, w, bias=b, act="silu", keep_prob=0.9, seed=1, offset=2)
    for _ in range(2):  # second call exercises the re-armed arrival counters
        out = kern.gemm(x.to(DEV), w.to(DEV), bias=b.to(DEV), act="silu", keep_prob=0.9, seed=1, offset=2, cfg=cfg,
                        splits=splits)
        _close(out, ref)
    acc_r = torch.full((M, N), 0.5)
    kern.gemm(x, w, out=acc_r, accumulate=True)
    acc_g = torch.full((M, N), 0.5, device=DEV)
    kern.gemm(x.to(DEV), w.to(DEV), out=acc_g, accumulate=True, cfg=cfg, splits=splits)
    _close(acc_g, acc_r, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("T,d", [(37, 64), (256, 512), (64, 1024), (2500, 512), (1536, 1024), (1030, 2048)])
def test_layernorm(T, d):
    x = _mk((T, d), torch.bfloat16, seed=31)
    gmm, bta = 1 + 0.1 * _mk((d,), torch.float32, seed=32), 0.1 * _mk((d,), torch.float32, seed=33)
    y_r, m_r, r_r = kern.layernorm_fwd(x, gmm, bta)
    y_g, m_g, r_g = kern.layernorm_fwd(x.to(DEV), gmm.to(DEV), bta.to(DEV))
    _close(y_g, y_r)
    _close(m_g, m_r, rtol=1e-5, atol=1e-5)
    _close(r_g, r_r, rtol=1e-4, atol=1e-4)
    dy, dres = _mk((T, d), torch.bfloat16, seed=34), _mk((T, d), torch.bfloat16, seed=35)
    dg_r, db_r, ds_r = torch.zeros(d), torch.zeros(d), torch.zeros(d)
    dx_r = kern.layernorm_bwd(dy, x, m_r, r_r, gmm, dg_r, db_r, dres=dres, dsum=ds_r)
    dg_g, db_g, ds_g = torch.zeros(d, device=DEV), torch.zeros(d, device=DEV), torch.zeros(d, device=DEV)
    dx_g = kern.layernorm_bwd(dy.to(DEV), x.to(DEV), m_g, r_g, gmm.to(DEV), dg_g, db_g, dres=dres.to(DEV),
                              dsum=ds_g)
    _close(dx_g, dx_r)
    _close(dg_g, dg_r, rtol=1e-3, atol=1e-3)
    _close(db_g, db_r, rtol=1e-3, atol=1e-3)
    # dsum = colsum of the kernel's own (bf16) dx output
    _close(ds_g, dx_g.float().sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("d", [512, 1024])
def test_layernorm_bwd_every_shape_variant(d):
    """Every (waves per workgroup, rows per wave) instantiation of ln_bwd, forced
    through the sweep knobs on a ragged row count, == the fp32 CPU reference."""
    from jax_distributed_tuts_amd.ops import _lib

    T = 333
    x = _mk((T, d), torch.bfloat16, seed=41)
    gmm = 1 + 0.1 * _mk((d,), torch.float32, seed=42)
    _, m_r, r_r = kern.layernorm_fwd(x, gmm, torch.zeros(d))
    dy, dres = _mk((T, d), torch.bfloat16, seed=43), _mk((T, d), torch.bfloat16, seed=44)
    dg_r, db_r = torch.zeros(d), torch.zeros(d)
    dx_r = kern.layernorm_bwd(dy, x, m_r, r_r, gmm, dg_r, db_r, dres=dres)
    lib = _lib.lib()
    try:
        for W, R in ((4, 1), (4, 2), (4, 4), (4, 8), (8, 1), (8, 2), (8, 4), (16, 1), (16, 2)):
            lib.jdt_ln_set_waves(W)
            lib.jdt_ln_set_rows(R)
            dg_g, db_g, ds_g = (torch.zeros(d, device=DEV) for _ in range(3))
            dx_g = kern.layernorm_bwd(dy.to(DEV), x.to(DEV), m_r.to(DEV), r_r.to(DEV), gmm.to(DEV), dg_g, db_g,
                                      dres=dres.to(DEV), dsum=ds_g)
            _close(dx_g, dx_r)
            _close(dg_g, dg_r, rtol=1e-3, atol=1e-3)
            _close(db_g, db_r, rtol=1e-3, atol=1e-3)
            _close(ds_g, dx_g.float().sum(0), rtol=1e-4, atol=1e-3)
    finally:
        lib.jdt_ln_set_waves(0)
        lib.jdt_ln_set_rows(0)


@pytest.mark.parametrize("B,S,H,Dh", [(2, 16, 4, 16), (2, 128, 8, 64), (1, 96, 2, 32)])
def test_attention_fwd_bwd(B, S, H, Dh):
    d = H * Dh
    qkv = _mk((B * S, 3 * d), torch.bfloat16, seed=41)
    o_r, p_r = kern.attention_fwd(qkv, B, S, H)
    o_g, p_g = kern.attention_fwd(qkv.to(DEV), B, S, H, impl="composed")  # GEMM + softmax kernels
    _close(o_g, o_r)
    _close(p_g, p_r)
    do = _mk((B * S, d), torch.bfloat16, seed=42)
    g_r = kern.attention_bwd(do, qkv, p_r, B, S, H)
    g_g = kern.attention_bwd(do.to(DEV), qkv.to(DEV), p_g, B, S, H)
    _close(g_g, g_r, rtol=3e-2, atol=3e-2)
    # flash path twice in a row: its persistent dQ workspace and tickets are left zeroed
    o_f, lse_f = kern.attention_fwd(qkv.to(DEV), B, S, H)
    g1 = kern.attention_bwd(do.to(DEV), qkv.to(DEV), lse_f, B, S, H, o=o_f)
    g2 = kern.attention_bwd(do.to(DEV), qkv.to(DEV), lse_f, B, S, H, o=o_f)
    assert torch.equal(g1, g2)
    _close(g1, g_r, rtol=3e-2, atol=3e-2)


def test_embedding_and_colsum():
    V, S, d, T = 100, 16, 64, 48
    wte, wpe = _mk((V, d), torch.bfloat16, seed=51), _mk((S, d), torch.bfloat16, seed=52)
    tok = torch.randint(0, V, (T,), generator=torch.Generator().manual_seed(5)).to(torch.int32)
    _close(kern.embed_fwd(tok.to(DEV), wte.to(DEV), wpe.to(DEV), S), kern.embed_fwd(tok, wte, wpe, S))
    dout = _mk((T, d), torch.bfloat16, seed=53)
    a_r, b_r = torch.zeros(V, d), torch.zeros(S, d)
    kern.embed_bwd(dout, tok, a_r, b_r, S)
    a_g, b_g = torch.zeros(V, d, device=DEV), torch.zeros(S, d, device=DEV)
    kern.embed_bwd(dout.to(DEV), tok.to(DEV), a_g, b_g, S)
    _close(a_g, a_r, rtol=1e-4, atol=1e-4)
    _close(b_g, b_r, rtol=1e-4, atol=1e-4)
    for M, N in ((T, d), (512, 1536), (77, 520), (1030, 2048)):
        x = _mk((M, N), torch.bfloat16, seed=54 + M)
        c_r = torch.ones(N)
        kern.colsum_(x, c_r)
        c_g = torch.ones(N, device=DEV)
        kern.colsum_(x.to(DEV), c_g)
        _close(c_g, c_r, rtol=1e-4, atol=1e-3)


def test_transformer_step_gpu_matches_cpu():
    from jax_distributed_tuts_amd.models.mlp import loss_and_grad
    from jax_distributed_tuts_amd.models.transformer import TransformerConfig, TransformerLM
    from jax_distributed_tuts_amd.parallel.pipeline_lm import lm_batch
    from jax_distributed_tuts_amd.utils.flat import FlatParams

    cfg = TransformerConfig(vocab_size=256, d_model=128, n_heads=4, d_ff=256, seq_len=32, n_layers=2)
    model = TransformerLM(cfg)
    b = lm_batch(cfg, 4, seed=2)
    res = {}
    for dev in ("cpu", DEV):
        P = FlatParams(model.param_specs(), device=dev).init_(0)
        m = torch.zeros(4, device=dev)
        loss_and_grad(model, P, b.inputs.to(dev), b.labels.to(dev), train=False, seed=0, offset=0, step=None,
                      metrics=m)
        res[dev] = (P.grad.cpu(), m.cpu())
    g_c, g_g = res["cpu"][0], res[DEV][0]
    assert float((g_g - g_c).norm() / g_c.norm()) < 3e-2
    _close(res[DEV][1], res["cpu"][1], rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("width", [(1024, 512), (1024, 256)])
def test_fused_mlp_input_width_1024(width):
    """The 2-layer fused engine at input width 1024 (16 backward chunks of 64 rows,
    csrc/mlp_fused.hip mlp2_kc): eager two-launch steps and captured run-ahead steps
    (one launch per step) == the generic-kernel path over the same rows."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    K, H = width
    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(128, K, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    out = {}
    for accum in ("fused", "kernel"):
        st = init_dp(Classifier(input_size=K, hidden_size=H), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, accum))
        for _ in range(2):
            tr.step(b)
        tr.capture(b, steps_per_graph=2)
        tr.run_steps(b, 4)
        tr.finalize()
        torch.cuda.synchronize()
        if accum == "kernel":
            assert tr.fused is not None and tr.fused.K == K and tr.fused.kc == 64 and tr.fused.ahead_ok
            assert tr._ahead is not None   # captured as run-ahead launches
        out[accum] = (st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()))
    assert out["kernel"][2] == out["fused"][2] == 6
    d = (out["kernel"][0] - out["fused"][0]).abs()
    assert float(d.max()) <= 2 * 1e-3 * 6 and float((d > 1e-4).float().mean()) < 5e-3, float(d.max())
    _close(out["kernel"][1], out["fused"][1], rtol=1e-3, atol=5e-2)


@pytest.mark.parametrize("fused_opt", ["1", "0"])
@pytest.mark.parametrize("rows", [128, 32, 16])
@pytest.mark.parametrize("layers", [2, 3, 4])
def test_fused_mlp_step_matches_generic(fused_opt, rows, layers, monkeypatch):
    """Whole-step fused kernels (mlp2_fwd/mlp2_bwd, optionally with AdamW in the
    epilogue) == the generic-kernel path over the same rows (same Philox dropout
    stream: row*H + col under (seed, step))."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    monkeypatch.setenv("JDT_FUSED_OPT", fused_opt)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(rows, 784, generator=g).to(DEV)
    y = torch.randint(0, 10, (rows,), generator=g).to(torch.int32).to(DEV)
    out = {}
    for accum in ("fused", "kernel"):
        st = init_dp(Classifier(num_layers=layers), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, accum))
        for _ in range(3):
            tr.step(Batch(x, y))
        tr.finalize()
        torch.cuda.synchronize()
        out[accum] = (st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()),
                      st.params.shadow.clone())
        if accum == "kernel":
            assert tr.fused is not None and tr.fused.fuse_opt == (fused_opt == "1")
    assert out["kernel"][2] == out["fused"][2] == 3
    d = (out["kernel"][0] - out["fused"][0]).abs()
    assert float(d.max()) <= 6e-3 and float((d > 1e-4).float().mean()) < 2e-3
    _close(out["kernel"][1], out["fused"][1], rtol=1e-3, atol=2e-2)
    sd = (out["kernel"][3].float() - out["fused"][3].float()).abs()
    assert float(sd.max()) <= 1e-2


@pytest.mark.parametrize("layers", [2, 4])
def test_fused_mlp_graph_capture(layers, monkeypatch):
    """Captured steps == eager steps with the same launch sequence (the run-ahead
    schedule, whose Z_0 summation order differs, has its own tests)."""
    monkeypatch.setenv("JDT_MLP2_AHEAD", "0")
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(0)
    x = torch.randn(128, 784, generator=g).to(DEV)
    y = torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV)
    res = []
    for graph in (False, True):
        st = init_dp(Classifier(num_layers=layers), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
        tr.step(Batch(x, y))
        if graph:
            tr.capture(Batch(x, y))
        for _ in range(6):
            tr.step(Batch(x, y))
        tr.finalize()
        torch.cuda.synchronize()
        res.append((st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item())))
    assert res[0][2] == res[1][2] == 7
    d = (res[0][0] - res[1][0]).abs()
    assert float(d.max()) <= 3e-3 and float((d > 1e-5).float().mean()) < 1e-3
    _close(res[1][1], res[0][1], rtol=1e-4, atol=1e-2)


def test_multi_step_graph_equals_single_steps():
    """A hipGraph holding 5 complete training steps == 5 single-step replays."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    res = []
    for spg in (1, 5):
        st = init_dp(Classifier(), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
        tr.step(b)
        tr.capture(b, steps_per_graph=spg)
        tr.run_steps(b, 12)
        tr.finalize()
        torch.cuda.synchronize()
        res.append((st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()), st.step))
    assert res[0][2] == res[1][2] == 13 and res[0][3] == res[1][3] == 13
    d = (res[0][0] - res[1][0]).abs()
    assert float(d.max()) <= 3e-3 and float((d > 1e-5).float().mean()) < 1e-3
    _close(res[1][1], res[0][1], rtol=1e-4, atol=1e-2)


def test_dp_scan_equals_loop_with_dropout():
    """accum="scan" (one captured minibatch step replayed per minibatch, device
    minibatch index) == the unrolled loop, dropout on (util.py:81-137 vs 41-78):
    same masks, eager and under the trainer's whole-step capture."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    res = {}
    for accum in ("loop", "scan"):
        st = init_dp(Classifier(), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, accum))
        for _ in range(3):
            tr.step(b)
        if accum == "scan":
            assert tr._scan is not None
        tr.capture(b)
        for _ in range(2):
            tr.step(b)
        tr.finalize()
        torch.cuda.synchronize()
        res[accum] = (st.params.master.clone(), tr.metrics.clone())
    # same dropout masks and minibatches; only fp32 atomic-order noise (bias colsums,
    # metric sums) -- a different mask stream moves most weights by >> 1e-5
    d = (res["loop"][0] - res["scan"][0]).abs()
    assert float(d.max()) <= 3e-3 and float((d > 1e-5).float().mean()) < 1e-3
    _close(res["scan"][1], res["loop"][1], rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("rows", [128, 32, 16])
def test_mlp2_loop_kernel_matches_two_launch(rows, monkeypatch):
    """The persistent n-step kernel (grid barriers, sc1 hand-offs) == the
    two-launch step, through the public multi-step graph path, and its barrier
    counter stays consistent across launches (eager launches after the graph)."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(rows, 784, generator=g).to(DEV),
              torch.randint(0, 10, (rows,), generator=g).to(torch.int32).to(DEV))
    res = {}
    for loop in ("0", "1"):
        monkeypatch.setenv("JDT_MLP2_LOOP", loop)
        st = init_dp(Classifier(), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
        tr.step(b)
        assert tr.fused.loop_ok == (loop == "1")
        tr.capture(b, steps_per_graph=5)
        tr.run_steps(b, 10)
        if loop == "1":
            assert tr.fused.run_loop(b, 3) and tr.fused.run_loop(b, 1)
        else:
            for _ in range(4):
                tr.fused.forward_backward(b)
        tr.finalize()
        torch.cuda.synchronize()
        res[loop] = (st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()),
                     st.params.shadow.clone())
        if loop == "1":
            w = tr.fused.loop_ws.cpu()
            assert int(w[2]) == 0 and int(w[0]) == int(w[1])   # no timeout; counter == next base
    assert res["0"][2] == res["1"][2] == 15
    d = (res["0"][0] - res["1"][0]).abs()
    assert float(d.max()) <= 3e-3 and float((d > 1e-5).float().mean()) < 1e-3
    _close(res["1"][1], res["0"][1], rtol=1e-4, atol=1e-2)
    sd = (res["0"][3].float() - res["1"][3].float()).abs()
    assert float(sd.max()) <= 1e-2


@pytest.mark.parametrize("rows", [128, 64, 32])
def test_mlp2_run_ahead_matches_two_launch(rows, monkeypatch):
    """One launch per step (step t's backward + AdamW + step t+1's forward, XCD-local
    column barriers) == two launches per step, through the multi-step graphs (cold
    with the prologue forward, then primed without it), 1-step primed graphs, and
    eager run-ahead launches mixed with two-launch steps (logits accumulators, step
    and launch counters stay consistent).  The run-ahead's Z1 sums 7 input-chunk
    partials instead of 8 wave partials, so agreement is to fp32 rounding."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(1)
    b = Batch(torch.randn(rows, 784, generator=g).to(DEV),
              torch.randint(0, 10, (rows,), generator=g).to(torch.int32).to(DEV))
    res = {}
    for ahead in ("0", "1"):
        monkeypatch.setenv("JDT_MLP2_AHEAD", ahead)
        st = init_dp(Classifier(), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
        tr.step(b)
        eng = tr.fused
        assert eng.ahead_ok == (ahead == "1")
        tr.capture(b, steps_per_graph=7)
        tr.run_steps(b, 14)          # cold 7-step graph, then the primed one
        tr.step(b)
        tr.step(b)                   # 1-step primed graphs
        eng.forward_backward(b)      # two launches: clears the primed state
        if ahead == "1":
            assert not eng.ahead_primed
            eng.run_ahead(b, 3)
            eng.run_ahead(b, 2, prologue=False)
        else:
            for _ in range(5):
                eng.forward_backward(b)
        eng.forward_backward(b)
        tr.finalize()
        torch.cuda.synchronize()
        res[ahead] = (st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()),
                      st.params.shadow.clone())
        if ahead == "1":
            zt = eng.ztick.cpu()
            nb = 512 // 16
            n = 7 + 7 + 1 + 1 + 3 + 2   # run-ahead launches
            assert int(zt[0]) == 0 and int(zt[1]) == 0 and int(zt[2]) == n   # ticket re-armed, no error, launches
            assert bool((zt[32:32 * (1 + nb)].view(nb, 32)[:, 0] == 7 * n).all())   # column barriers: 7 per launch
            tiles = zt[32 * (1 + nb):].view(8, 32)[:, :28]
            assert bool((tiles == n).all())   # every tile ran exactly once per launch
    assert res["0"][2] == res["1"][2] == 24
    d = (res["0"][0] - res["1"][0]).abs()
    assert float(d.max()) <= 3e-3 and float((d > 1e-5).float().mean()) < 1e-2
    _close(res["1"][1], res["0"][1], rtol=1e-3, atol=5e-2)
    sd = (res["0"][3].float() - res["1"][3].float()).abs()
    assert float(sd.max()) <= 1e-2


@pytest.mark.parametrize("layers", [2, 4])
def test_fsdp_fused_kernels_match_generic(layers):
    """FSDP (world 1) with the fused classifier kernels on the gathered buffer ==
    FSDP with the generic kernels (gather/scatter once).  Dropout off: the generic
    path indexes the dropout stream per minibatch, the fused one per device pass."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    res = []
    for fused in (False, True):
        st = init_fsdp(Classifier(dropout_rate=0.0, num_layers=layers), adamw(1e-3), 69, DEV, None, "data", 16)
        tr = FSDPTrainer(st, None, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=fused,
                                              fused_loop=False))
        for _ in range(3):
            tr.step(b)
        torch.cuda.synchronize()
        res.append((st.params.master.clone(), tr.metrics.clone()))
        if fused:
            assert tr.fused is not None
    d = (res[0][0] - res[1][0]).abs()
    assert float(d.max()) <= 6e-3 and float((d > 1e-4).float().mean()) < 2e-3
    _close(res[1][1], res[0][1], rtol=1e-3, atol=2e-2)


@pytest.mark.parametrize("layers", [2, 4])
def test_fsdp_fused_loop_matches_generic_loop(layers):
    """The reference's per-minibatch FSDP schedule (gather / fwd+bwd / reduce-scatter
    every minibatch, param_sharding.py) on the fused md kernels (FSDPConfig.fused_loop)
    == the same schedule on the generic GEMM chain, dropout ON (both draw stream
    (i << 16) + (l << 1) at the step counter) and a scale-revealing SGD, eager and
    replayed from a multi-step hipGraph."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.train_state import Batch, sgd

    g = torch.Generator().manual_seed(0)
    b = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    res = []
    for fl in (False, True):
        st = init_fsdp(Classifier(num_layers=layers), sgd(0.05), 69, DEV, None, "data", 16)
        tr = FSDPTrainer(st, None, FSDPConfig(4, 16, "data", fused_loop=fl))
        tr.step(b)
        tr.capture(b, steps_per_graph=2)
        tr.run_steps(b, 4)
        torch.cuda.synchronize()
        assert (tr._loop_engine is not None) == fl
        res.append((st.params.master.clone(), tr.metrics.clone()))
    d = (res[0][0] - res[1][0]).abs()
    print(f"[fsdp loop L{layers}] max |dp| {float(d.max()):.3e}")
    assert float(d.max()) <= 2e-3 * float(res[0][0].abs().max())
    _close(res[1][1], res[0][1], rtol=1e-3, atol=2e-2)


def test_fsdp_run_ahead_matches_two_launch(monkeypatch):
    """FSDP at N = 1 (the DP engine on whole-leaf shards) through captured graphs:
    run-ahead (one launch per step) == two launches per step, to fp32 rounding."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(2)
    b = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    res = {}
    for ahead in ("0", "1"):
        monkeypatch.setenv("JDT_MLP2_AHEAD", ahead)
        st = init_fsdp(Classifier(), adamw(1e-4), 6969, DEV, None, "data", 16)
        tr = FSDPTrainer(st, None, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=True))
        tr.step(b)
        tr.capture(b, steps_per_graph=5)
        assert (tr._ahead is not None) == (ahead == "1")
        tr.run_steps(b, 10)
        tr.step(b)
        tr.finalize() if hasattr(tr, "finalize") else tr.fused.finalize()
        torch.cuda.synchronize()
        res[ahead] = (st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()))
    assert res["0"][2] == res["1"][2] == 12
    d = (res["0"][0] - res["1"][0]).abs()
    assert float(d.max()) <= 3e-3 and float((d > 1e-5).float().mean()) < 1e-2
    _close(res["1"][1], res["0"][1], rtol=1e-3, atol=5e-2)


@pytest.mark.parametrize("B,S,H", [(2, 128, 8), (1, 96, 2), (2, 200, 4), (1, 64, 1)])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_fwd_bwd(B, S, H, causal):
    """Fused flash kernels (Dh=64) vs the torch reference (P rounded to bf16 like the kernels)."""
    d = H * 64
    qkv = _mk((B * S, 3 * d), torch.bfloat16, seed=61)
    Dh = 64
    q, k, v = qkv.float().view(B, S, 3, H, Dh).permute(2, 0, 3, 1, 4)
    s = torch.matmul(q, k.transpose(-1, -2)) / 8.0
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool), 1), float("-inf"))
    p = torch.softmax(s, -1)
    o_ref = torch.matmul(p, v).permute(0, 2, 1, 3).reshape(B * S, d)
    o_g, lse = kern.attention_fwd(qkv.to(DEV), B, S, H, causal=causal)
    assert lse.shape == (B * H, S)
    _close(o_g, o_ref, rtol=2e-2, atol=2e-2)
    _close(lse.view(B, H, S), torch.logsumexp(s, -1), rtol=1e-3, atol=1e-3)
    do = _mk((B * S, d), torch.bfloat16, seed=62)
    # fp32 autograd reference
    qkv_r = qkv.float().clone().requires_grad_()
    q2, k2, v2 = qkv_r.view(B, S, 3, H, Dh).permute(2, 0, 3, 1, 4)
    s2 = torch.matmul(q2, k2.transpose(-1, -2)) / 8.0
    if causal:
        s2 = s2.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool), 1), float("-inf"))
    o2 = torch.matmul(torch.softmax(s2, -1), v2).permute(0, 2, 1, 3).reshape(B * S, d)
    (o2 * do.float()).sum().backward()
    db = torch.full((3 * d,), 0.5, device=DEV)
    g = kern.attention_bwd(do.to(DEV), qkv.to(DEV), lse, B, S, H, o=o_g, causal=causal, dbias=db)
    _close(g, qkv_r.grad, rtol=3e-2, atol=3e-2)
    _close(db, g.float().sum(0) + 0.5, rtol=1e-4, atol=1e-3)  # fused QKV bias gradient
    # composed (GEMM + softmax kernels) path agrees with the fused one
    o_c, P = kern.attention_fwd(qkv.to(DEV), B, S, H, causal=causal, impl="composed")
    _close(o_c, o_g, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,K,N,act", [(2048, 512, 1536, "none"), (512, 512, 2048, "gelu"), (256, 512, 1536, "none"),
                                        (96, 1024, 128, "gelu"), (40, 512, 64, "none")])
def test_ln_gemm_matches_layernorm_then_gemm(M, K, N, act):
    """LayerNorm fused into the GEMM A operand (gemm_ln_kernel) == ln_fwd + gemm:
    LN(x) and its statistics bit-identical, C within bf16 rounding (M = 40 takes the
    two-launch fallback)."""
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(M, K, generator=g) * 2 + 0.5).to(torch.bfloat16).to(DEV)
    gamma = (1 + 0.1 * torch.randn(K, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(K, generator=g)).to(DEV)
    w = (torch.randn(K, N, generator=g) / K ** 0.5).to(torch.bfloat16).to(DEV)
    bias = (0.1 * torch.randn(N, generator=g)).to(torch.bfloat16).to(DEV)
    from jax_distributed_tuts_amd.ops import _lib

    y_r, m_r, r_r = kern.layernorm_fwd(x, gamma, beta, 1e-6)
    z_r = torch.empty(M, N, dtype=torch.bfloat16, device=DEV) if act != "none" else None
    c_r = kern.gemm(y_r, w, bias=bias, act=act, z_out=z_r)
    try:
        for cfg in (0, 1, 2, 3, 4):  # heuristic (may fall back) and every fused tile
            if cfg in (2, 4) and M % 64:
                continue
            _lib.lib().jdt_gemm_ln_set_cfg(cfg)
            z = torch.empty(M, N, dtype=torch.bfloat16, device=DEV) if act != "none" else None
            c, y, mean, rstd = kern.ln_gemm(x, gamma, beta, w, eps=1e-6, bias=bias, act=act, z_out=z)
            torch.cuda.synchronize()
            assert torch.equal(y, y_r) and torch.equal(mean, m_r) and torch.equal(rstd, r_r), cfg
            _close(c, c_r, rtol=1e-2, atol=1e-2)
            if z is not None:
                _close(z, z_r, rtol=1e-2, atol=1e-2)
    finally:
        _lib.lib().jdt_gemm_ln_set_cfg(0)
    # against fp32 torch
    ref = torch.nn.functional.layer_norm(x.float(), (K,), gamma, beta, 1e-6).to(torch.bfloat16).float() @ w.float()
    ref = ref + bias.float()
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    _close(c, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("T,S,d,N", [(2048, 128, 512, 1536), (256, 128, 512, 1536), (333, 111, 1024, 128),
                                     (96, 32, 2048, 64)])
def test_embedding_fused_layernorm(T, S, d, N):
    """layernorm_fwd(embed=) / ln_gemm(embed=) (jdt_ln_fwd_embed: the token + position
    embedding built inside the LN launch) == embed_fwd then layernorm_fwd: the embedding
    written to x, LN(x) and its statistics bit-identical; T = 256 takes the fused
    LN-GEMM route (embedding launched apart), T = 2048 the LN-apart one."""
    V = 300
    gen = torch.Generator().manual_seed(8)
    wte = (torch.randn(V, d, generator=gen) * 0.5).to(torch.bfloat16).to(DEV)
    wpe = (torch.randn(S, d, generator=gen) * 0.5).to(torch.bfloat16).to(DEV)
    tok = torch.randint(0, V, (T,), generator=gen).to(torch.int32).to(DEV)
    gamma = (1 + 0.1 * torch.randn(d, generator=gen)).to(DEV)
    beta = (0.1 * torch.randn(d, generator=gen)).to(DEV)
    e_r = kern.embed_fwd(tok, wte, wpe, S)
    y_r, m_r, r_r = kern.layernorm_fwd(e_r, gamma, beta, 1e-6)
    x = torch.full((T, d), float("nan"), dtype=torch.bfloat16, device=DEV)
    y, mean, rstd = kern.layernorm_fwd(x, gamma, beta, 1e-6, embed=(tok, wte, wpe, S))
    torch.cuda.synchronize()
    assert torch.equal(x, e_r) and torch.equal(y, y_r) and torch.equal(mean, m_r) and torch.equal(rstd, r_r)
    # CPU oracle of the embedding itself
    _close(x, kern.embed_fwd(tok.cpu(), wte.cpu(), wpe.cpu(), S), rtol=0, atol=0)
    w = (torch.randn(d, N, generator=gen) / d ** 0.5).to(torch.bfloat16).to(DEV)
    c_r = kern.gemm(y_r, w)
    x2 = torch.full((T, d), float("nan"), dtype=torch.bfloat16, device=DEV)
    c, y2, m2, r2 = kern.ln_gemm(x2, gamma, beta, w, eps=1e-6, embed=(tok, wte, wpe, S))
    torch.cuda.synchronize()
    assert torch.equal(x2, e_r) and torch.equal(y2, y_r) and torch.equal(m2, m_r) and torch.equal(r2, r_r)
    _close(c, c_r, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,S,H", [(2, 128, 8), (3, 96, 2), (1, 40, 3), (2, 17, 1), (1, 128, 1)])
@pytest.mark.parametrize("causal", [True, False])
def test_attn128_vs_autograd_and_flash(B, S, H, causal):
    """S <= 128 attention kernels (csrc/attn128.hip) against an fp32 autograd oracle,
    the tile-streaming flash kernels, and themselves (bitwise reproducible)."""
    from jax_distributed_tuts_amd.ops import _lib

    d, Dh = H * 64, 64
    qkv = _mk((B * S, 3 * d), torch.bfloat16, seed=71)
    do = _mk((B * S, d), torch.bfloat16, seed=72)
    qkv_r = qkv.float().clone().requires_grad_()
    q2, k2, v2 = qkv_r.view(B, S, 3, H, Dh).permute(2, 0, 3, 1, 4)
    s2 = torch.matmul(q2, k2.transpose(-1, -2)) / 8.0
    if causal:
        s2 = s2.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool), 1), float("-inf"))
    o2 = torch.matmul(torch.softmax(s2, -1), v2).permute(0, 2, 1, 3).reshape(B * S, d)
    (o2 * do.float()).sum().backward()
    res = {}
    try:
        for impl in (1, 0, 1):
            _lib.lib().jdt_flash_set_attn128(impl)
            o_g, lse = kern.attention_fwd(qkv.to(DEV), B, S, H, causal=causal)
            db = torch.full((3 * d,), 0.25, device=DEV)
            g = kern.attention_bwd(do.to(DEV), qkv.to(DEV), lse, B, S, H, o=o_g, causal=causal, dbias=db)
            torch.cuda.synchronize()
            if impl in res:  # second attn128 run: bitwise identical (fixed order, no atomics on dQ)
                assert torch.equal(o_g, res[impl][0]) and torch.equal(g, res[impl][2])
            res[impl] = (o_g, lse, g, db)
    finally:
        _lib.lib().jdt_flash_set_attn128(1)
    o_n, lse_n, g_n, db_n = res[1]
    _close(o_n, o2.detach(), rtol=2e-2, atol=2e-2)
    _close(lse_n.view(B, H, S), torch.logsumexp(s2.detach(), -1), rtol=1e-3, atol=1e-3)
    _close(g_n, qkv_r.grad, rtol=3e-2, atol=3e-2)
    _close(db_n, g_n.float().sum(0) + 0.25, rtol=1e-4, atol=1e-3)
    # relative L2 error per q / k / v block, against the old kernels' error
    for part in range(3):
        ref = qkv_r.grad.view(B * S, 3, d)[:, part].float().cpu()
        e_new = float((g_n.view(B * S, 3, d)[:, part].float().cpu() - ref).norm() / ref.norm().clamp_min(1e-12))
        e_old = float((res[0][2].view(B * S, 3, d)[:, part].float().cpu() - ref).norm() / ref.norm().clamp_min(1e-12))
        assert e_new < 1.5 * e_old + 2e-3, (part, e_new, e_old)
    _close(o_n, res[0][0], rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("fused", [True, False])
def test_fsdp_graph_replay_matches_eager(fused):
    """FSDP (world 1) captured as single- and multi-step hipGraphs == eager steps."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(3)
    b = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    res = []
    for graph in (False, True):
        st = init_fsdp(Classifier(), adamw(1e-3), 69, DEV, None, "data", 16)
        tr = FSDPTrainer(st, None, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=fused))
        tr.step(b)
        if graph:
            tr.capture(b, steps_per_graph=3)
            tr.run_steps(b, 7)
        else:
            for _ in range(7):
                tr.step(b)
        torch.cuda.synchronize()
        res.append((st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()), st.step))
    assert res[0][2] == res[1][2] == 8 and res[0][3] == res[1][3] == 8
    # fp32 atomics (split-K partial logits) make runs differ in the last bits; Adam can
    # turn that into an lr-sized move on a ~0 gradient, so bound the fraction
    d = (res[1][0] - res[0][0]).abs()
    assert float(d.max()) <= 2 * 1e-3 * 8 and float((d > 5e-5).float().mean()) < 2e-3
    torch.testing.assert_close(res[1][1], res[0][1], rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,D_out", [(256, 384), (32, 384), (96, 384), (256, 2048), (64, 1024)])
def test_gemm_group_matches_individual(M, D_out):
    """A layer's dW (km x kn, fp32 accumulate; K = M rows, a 32-deep tail tile when
    M % 64 == 32) and dX (mk x nk with act' * mask + dbias epilogue; K = D_out,
    split-K inside the group when >= 1024) in one grouped launch == the same GEMMs
    launched one by one; a non-eligible member falls back to individual launches."""
    D_in = 512
    h = _mk((M, D_in), torch.bfloat16, seed=71).to(DEV)
    dz = _mk((M, D_out), torch.bfloat16, seed=72).to(DEV)
    w = (_mk((D_in, D_out), torch.float32, seed=73) * 0.05).to(torch.bfloat16).to(DEV)
    z = _mk((M, D_in), torch.bfloat16, seed=74).to(DEV)
    outs = []
    for grouped in (False, True):
        gW = torch.full((D_in, D_out), 0.25, device=DEV)
        db = torch.zeros(D_in, device=DEV)
        dx = torch.empty(M, D_in, dtype=torch.bfloat16, device=DEV)

        def body():
            kern.gemm(h, dz, a_layout="km", b_layout="kn", out=gW, accumulate=True)
            kern.gemm(dz, w, b_layout="nk", out=dx, z_in=z, act_bwd="silu", keep_prob=0.9, seed=5, offset=9,
                      dbias=db)
        if grouped:
            with kern.gemm_group():
                body()
        else:
            body()
        torch.cuda.synchronize()
        outs.append((gW.clone(), dx.clone(), db.clone()))
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=1e-5, atol=1e-5)
    # dX: same MFMA order when both launches use the DMA path; the register path
    # (ungrouped, small M) may round differently in the last bf16 bit
    torch.testing.assert_close(outs[1][1].float(), outs[0][1].float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(outs[1][2], outs[0][2], rtol=1e-4, atol=1e-3)
    # ineligible shape inside a group: launched individually, same result as plain
    a, b = _mk((48, 24), torch.bfloat16, seed=75), _mk((24, 40), torch.bfloat16, seed=76)
    ref = kern.gemm(a, b, out_dtype=torch.float32)
    with kern.gemm_group():
        o1 = kern.gemm(a.to(DEV), b.to(DEV), out_dtype=torch.float32)
        o2 = kern.gemm(h, dz, a_layout="km", b_layout="kn", out_dtype=torch.float32)
    _close(o1, ref, rtol=1e-3, atol=1e-3)
    _close(o2, kern.gemm(h.cpu(), dz.cpu(), a_layout="km", b_layout="kn", out_dtype=torch.float32),
           rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("model", ["mlp", "transformer"])
def test_single_stage_pipeline_merge_gpu(model):
    """GPipe with one stage: microbatches merged into one pass (PipeConfig.merge_single_stage)
    == the microbatch loop on the GPU kernels (dropout off for the MLP; the
    transformer has none)."""
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline, lm_batch
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch

    mesh = Mesh({"data": 1, "pipe": 1})
    res = []
    for merge in (False, True):
        if model == "mlp":
            cfg = dp_config()
            tr = build_mlp_pipeline(cfg, mesh, DEV, 3, dropout_rate=0.0, num_microbatches=4, merge_single_stage=merge)
            b = synthetic_batch(cfg, 70)
        else:
            tr, lcfg = build_lm_pipeline(mesh, DEV, num_microbatches=4, merge_single_stage=merge)
            b = lm_batch(lcfg, global_batch=8, seed=1)
        if not merge:
            tr.cfg.layer_major_single_stage = False  # the real per-microbatch passes
        b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
        for _ in range(3):
            tr.step(b)
        torch.cuda.synchronize()
        res.append((tr.state.params.master.clone(), tr.metrics.clone()))
    d = (res[0][0] - res[1][0]).abs()
    assert float(d.max()) <= 6e-3 and float((d > 1e-4).float().mean()) < 5e-2
    _close(res[1][1], res[0][1], rtol=2e-3, atol=5e-2)


@pytest.mark.parametrize("graph", [False, True])
def test_overlapped_adamw_equals_single_launch(graph, monkeypatch):
    """One-stage transformer LM (layer-major): AdamW forked layer by layer onto a side
    stream during the backward (ops.kernels.OverlappedAdamW) == one AdamW launch after
    it (same per-element arithmetic, same step) to the step's own run-to-run noise --
    eager and captured into multi-step hipGraphs (the fork/join become graph
    branches).  A race (a layer updated before its last gradient contribution)
    would show as an error far above that noise."""
    from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline, lm_batch
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.train_state import Batch

    mesh = Mesh({"data": 1, "pipe": 1})
    res = {}
    for ov in ("0", "1", "0b"):
        monkeypatch.setenv("JDT_OVERLAP_OPT", ov[0])
        monkeypatch.setenv("JDT_LM_FUSED_OPT", "0")  # the in-epilogue AdamW would take precedence
        monkeypatch.setenv("JDT_MB_STREAMS", "1")    # layer-major (concurrent microbatch passes otherwise)
        # the weight GEMMs inline in every variant: the comparison isolates where AdamW runs
        # (the one-launch W pass, which the overlapped form cannot use, sums in another order)
        monkeypatch.setenv("JDT_WPASS_ONE", "0")
        tr, lcfg = build_lm_pipeline(mesh, DEV, num_microbatches=4)
        b = lm_batch(lcfg, global_batch=8, seed=1)
        b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
        tr.step(b)
        assert bool(getattr(tr, "_ov_opt", None)) == (ov == "1")
        if graph:
            tr.capture(b, steps_per_graph=3)
            tr.run_steps(b, 6)
        else:
            for _ in range(3):
                tr.step(b)
        torch.cuda.synchronize()
        st = tr.state
        res[ov] = (st.params.master.clone(), st.params.shadow.clone(), st.opt_state["m"].clone(),
                   tr.metrics.clone(), int(st.opt_state["count"].item()))
    assert res["0"][4] == res["1"][4] == res["0b"][4]
    # The step is not bitwise reproducible (fp32 atomics in the LN / embedding / CE
    # reductions), and AdamW turns tiny gradient differences into lr-sized updates
    # where g ~ 0.  So compare the FRACTION of parameters that moved apart: a race
    # (a layer updated before its last gradient contribution, or a lower layer's
    # backward reading already-updated weights) shifts whole layers, the noise only
    # scattered elements.  The loss sums must agree closely.
    def frac(a, c):
        return float(((a - c).abs() > 1e-5).float().mean())

    noise, diff = frac(res["0"][0], res["0b"][0]), frac(res["0"][0], res["1"][0])
    print(f"params differing > 1e-5: run-to-run {noise:.2e}, overlapped {diff:.2e}")
    # a race moves whole weight matrices (each block's 4 kernels are ~24 % of the stage);
    # a run whose atomics happened to be order-identical (noise 0) still leaves ~1 % of
    # near-zero-gradient elements apart once the overlap reorders the reductions
    assert diff <= 4 * noise + 0.03, (diff, noise)
    loss = [float(r[3][0]) for r in (res["0"], res["1"], res["0b"])]
    assert abs(loss[1] - loss[0]) <= 1e-3 * abs(loss[0]) + 4 * abs(loss[2] - loss[0]), loss


@pytest.mark.parametrize("layers,rows", [(4, 128), (3, 64), (4, 32)])
def test_deep_run_ahead_matches_two_launch(layers, rows, monkeypatch):
    """Deep MLP (FusedMLPDeep): the layer-0 backward also running layer 0's forward of
    the next step (md_bwd AHEAD) == the plain launch sequence, through cold / primed
    multi-step graphs, 1-step graphs and eager launches mixed with plain steps."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(3)
    b = Batch(torch.randn(rows, 784, generator=g).to(DEV),
              torch.randint(0, 10, (rows,), generator=g).to(torch.int32).to(DEV))
    res = {}
    for ahead in ("0", "1"):
        monkeypatch.setenv("JDT_MLP2_AHEAD", ahead)
        st = init_dp(Classifier(num_layers=layers), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
        tr.step(b)
        eng = tr.fused
        assert eng.ahead_ok == (ahead == "1")
        tr.capture(b, steps_per_graph=5)
        tr.run_steps(b, 10)
        tr.step(b)
        eng.forward_backward(b)
        if ahead == "1":
            eng.run_ahead(b, 2)
            eng.run_ahead(b, 1, prologue=False)
        else:
            for _ in range(3):
                eng.forward_backward(b)
        eng.forward_backward(b)
        tr.finalize()
        torch.cuda.synchronize()
        res[ahead] = (st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()))
        if ahead == "1":
            zt = eng.ztick.cpu()
            n = 5 + 5 + 1 + 2 + 1   # run-ahead launches
            assert int(zt[1]) == 0 and int(zt[2]) == n, zt[:3]
            assert bool((zt[32:32 * 33].view(32, 32)[:, 0] == 7 * n).all())
            assert bool((zt[32 * 33:].view(8, 32)[:, :28] == n).all())
        if ahead == "1":
            # the run-ahead's layer-0 forward of the next step == md_fwd of that step
            import ctypes

            from jax_distributed_tuts_amd.ops import _lib

            eng.run_ahead(b, 1)
            torch.cuda.synchronize()
            h_a, g_a = eng.Hs[0].clone(), eng.G[0].clone()
            _lib.check(_lib.lib().jdt_md_layer(ctypes.byref(eng._args[0][0]), 0, 0, _lib.stream_ptr()), "md_fwd")
            torch.cuda.synchronize()
            dh = (h_a.float() - eng.Hs[0].float()).abs()
            assert float((dh > 0).float().mean()) < 0.02 and float(dh.max()) <= 0.05, float(dh.max())
            dg = (g_a - eng.G[0]).abs()
            assert float((dg > 1e-3).float().mean()) < 0.02
    assert res["0"][2] == res["1"][2] == 17
    # 4 layers of AdamW over 17 steps amplify the Z_0 summation-order difference into
    # many tiny parameter differences; the forward check above is the precise one
    d = (res["0"][0] - res["1"][0]).abs()
    assert float(d.max()) <= 3e-3
    _close(res["1"][1], res["0"][1], rtol=1e-3, atol=5e-2)


def test_pipeline_single_stage_run_ahead(monkeypatch):
    """One-stage GPipe on the deep fused engine (per-microbatch dropout streams,
    mb_rows): run-ahead graphs == the plain launch sequence, and the run-ahead's
    layer-0 forward (H_0 / G_0, per-microbatch masks) == md_fwd of the same step."""
    import ctypes

    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.ops import _lib
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch

    mesh = Mesh({"data": 1, "pipe": 1})
    monkeypatch.setenv("JDT_MLP2_AHEAD_MB", "1")   # opt-in for per-microbatch dropout streams
    res = {}
    for ahead in ("0", "1"):
        monkeypatch.setenv("JDT_MLP2_AHEAD", ahead)
        cfg = dp_config()
        tr = build_mlp_pipeline(cfg, mesh, DEV, 8, num_microbatches=4)
        b = synthetic_batch(cfg, 70)
        b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
        tr.step(b)
        eng = tr.deep_engine
        assert eng is not None and eng.mb_rows > 0 and eng.ahead_ok == (ahead == "1")
        tr.capture(b, steps_per_graph=3)
        tr.run_steps(b, 6)
        tr.step(b)
        tr.finalize()
        torch.cuda.synchronize()
        res[ahead] = (tr.state.params.master.clone(), tr.metrics.clone(), int(tr.state.opt_state["count"].item()))
        if ahead == "1":
            assert int(eng.ztick[1].item()) == 0
            eng.run_ahead(b, 1)
            torch.cuda.synchronize()
            h_a, g_a = eng.Hs[0].clone(), eng.G[0].clone()
            _lib.check(_lib.lib().jdt_md_layer(ctypes.byref(eng._args[0][0]), 0, 0, _lib.stream_ptr()), "md_fwd")
            torch.cuda.synchronize()
            dh = (h_a.float() - eng.Hs[0].float()).abs()
            assert float((dh > 0).float().mean()) < 0.02 and float(dh.max()) <= 0.05, float(dh.max())
            assert float(((g_a - eng.G[0]).abs() > 1e-3).float().mean()) < 0.02
    assert res["0"][2] == res["1"][2] == 8
    assert float((res["0"][0] - res["1"][0]).abs().max()) <= 3e-3
    _close(res["1"][1], res["0"][1], rtol=1e-3, atol=5e-2)


def test_deep_run_ahead_mb_streams_20_steps(monkeypatch):
    """JDT_MLP2_AHEAD_MB (run-ahead with per-microbatch dropout streams, one-stage GPipe
    on the deep engine) over 20 captured steps at keep 0.5, against the plain launch
    sequence: AdamW with b1 = b2 = 0 and eps = 10 makes every update
    g / (|g| + 10), proportional to that step's gradient, so the 20-step displacement of
    every leaf compares like a gradient (relative L2 error and least-squares scale).  A
    mask drawn from the wrong microbatch / step stream at keep 0.5 changes half of a
    layer's units: far outside bf16 noise."""
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    from .oracle import check_grad

    mesh = Mesh({"data": 1, "pipe": 1})
    monkeypatch.setenv("JDT_MLP2_AHEAD_MB", "1")
    res = {}
    for ahead in ("0", "1"):
        monkeypatch.setenv("JDT_MLP2_AHEAD", ahead)
        cfg = dp_config()
        tr = build_mlp_pipeline(cfg, mesh, DEV, 4, dropout_rate=0.5, num_microbatches=4,
                                tx=adamw(0.01, b1=0.0, b2=0.0, eps=10.0, weight_decay=0.0))
        b = synthetic_batch(cfg, 70)
        b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
        p0 = {k: v.detach().clone().cpu() for k, v in tr.state.params.state_dict().items()}
        tr.step(b)
        eng = tr.deep_engine
        assert eng is not None and eng.mb_rows > 0 and eng.ahead_ok == (ahead == "1")
        tr.capture(b, steps_per_graph=5)
        tr.run_steps(b, 15)
        for _ in range(4):
            tr.step(b)
        tr.finalize()
        torch.cuda.synchronize()
        assert int(tr.state.opt_state["count"].item()) == 20
        if ahead == "1":
            assert int(eng.ztick[1].item()) == 0
        res[ahead] = {k: (p0[k].double() - v.detach().cpu().double()) for k, v in tr.state.params.state_dict().items()}
    for k in res["0"]:
        check_grad(res["1"][k], res["0"][k], f"20-step displacement {k}")


@pytest.mark.parametrize("strategy", ["dp", "fsdp"])
def test_set_batch_after_capture_matches_eager(strategy):
    """New data for captured graphs: a step on other tensors raises (the graphs read the
    captured ones), ``set_batch`` copies the data in and restarts the run-ahead cold (its
    next forward was computed from the old contents) -- equal to eager steps on A, A, B, B."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(11)
    A = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    B = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    res = []
    for graph in (False, True):
        if strategy == "dp":
            st = init_dp(Classifier(), adamw(1e-3), 69, DEV)
            tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
        else:
            st = init_fsdp(Classifier(), adamw(1e-3), 69, DEV, None, "data", 16)
            tr = FSDPTrainer(st, None, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=True))
        a = Batch(A.inputs.clone(), A.labels.clone())   # the captured tensors (set_batch overwrites them)
        tr.step(a)
        if graph:
            tr.capture(a)
        tr.step(a)
        if graph:
            with pytest.raises(ValueError):
                tr.step(B)
            tr.set_batch(B)
            tr.step(a)
            tr.step(a)
        else:
            tr.step(B)
            tr.step(B)
        tr.finalize()
        torch.cuda.synchronize()
        res.append((st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item())))
    assert res[0][2] == res[1][2] == 4
    d = (res[0][0] - res[1][0]).abs()
    assert float(d.max()) <= 3e-3 and float((d > 1e-5).float().mean()) < 1e-3, (float(d.max()), float((d > 1e-5).float().mean()))
    _close(res[1][1], res[0][1], rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("layers,rows", [(4, 128), (3, 64), (4, 32)])
def test_deep_dz_split_bitwise(layers, rows, monkeypatch):
    """md_bwd dZ split (MdArgs::dzs: the K-chunk workgroups of a column block each
    compute 1/NCH of dZ_i's rows and exchange them through a per-block counter) ==
    every workgroup computing all rows, bit for bit: deterministic mode (ordered
    partial logits, no fp32 atomics), 3 eager steps of the deep engine; and the
    barrier's error word stays clear."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(5)
    b = Batch(torch.randn(rows, 784, generator=g).to(DEV), torch.randint(0, 10, (rows,), generator=g).to(torch.int32).to(DEV))
    monkeypatch.setenv("JDT_DETERMINISTIC", "1")
    res = {}
    for dzs in ("1", "0"):
        monkeypatch.setenv("JDT_MD_DZS", dzs)
        st = init_dp(Classifier(num_layers=layers), adamw(1e-3), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
        for _ in range(3):
            tr.step(b)
        eng = tr.fused
        assert eng.dzs_ok == (dzs == "1")
        assert eng.dzs_error() == 0
        tr.finalize()
        torch.cuda.synchronize()
        res[dzs] = (st.params.master.clone(), tr.metrics.clone())
    assert torch.equal(res["1"][0], res["0"][0])
    assert torch.equal(res["1"][1], res["0"][1])


def test_fused_sgd_matches_mode0_sgd(monkeypatch):
    """Momentum-free SGD fused into mlp2_bwd's epilogue (opt_sgd, incl. the run-ahead
    graphs) == mode 0 (plain-stored grads) + the standalone SGD kernel.  SGD moves
    parameters linearly in the gradient, so the two agree to fp32 rounding."""
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.utils.train_state import Batch, sgd

    g = torch.Generator().manual_seed(4)
    b = Batch(torch.randn(128, 784, generator=g).to(DEV), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    monkeypatch.setenv("JDT_FUSED_SGD", "1")
    res = {}
    for fused in ("0", "1"):
        monkeypatch.setenv("JDT_FUSED_OPT", fused)
        st = init_dp(Classifier(), sgd(0.05, weight_decay=1e-4), 69, DEV)
        tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
        tr.step(b)
        assert tr.fused.fuse_opt == (fused == "1") and tr.fused.opt_sgd
        tr.capture(b, steps_per_graph=5)
        tr.run_steps(b, 10)
        tr.step(b)
        tr.finalize()
        torch.cuda.synchronize()
        res[fused] = (st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item()),
                      st.params.shadow.clone())
    assert res["0"][2] == res["1"][2] == 12
    d = (res["0"][0] - res["1"][0]).abs()
    assert float(d.max()) <= 1e-4, float(d.max())
    _close(res["1"][1], res["0"][1], rtol=1e-3, atol=5e-2)
    assert float((res["0"][3].float() - res["1"][3].float()).abs().max()) <= 1e-2
