"""The persistent run-ahead launch (ops/csrc/mlp_fused.hip mlp2_pst_kernel): n >= 2
headline steps in ONE launch, each workgroup's AdamW state in registers across them and an
XCD-hierarchical grid barrier between steps, against the same steps as n run-ahead
launches (JDT_MLP2_PST=0) -- through the multi-step graphs (cold, then primed), 1-step
graphs, eager run-ahead calls and two-launch steps mixed in (logits accumulators, step,
launch and barrier counters stay consistent).  Same arithmetic in the same order except the
forward's fp32 logits atomics (32 column-block partials per logit, summed in arrival order
in BOTH forms), so the two agree to that rounding: usually bit-identical at 32 / 64 / 128
rows, but a different arrival order in either run perturbs a logit by ~1 ulp and AdamW
carries it on (m / sqrt(v) normalises the perturbation, it does not shrink it): one run
of 128 rows gave 99 % of the parameters different, median tiny, max |dp| 7.3e-6 = 6e-5 x
scale.  So the bounds are on the bulk: median |d| <= 1e-5 x scale and the 99.9th percentile
<= 1e-4 x scale.  A lost or doubly applied gradient tile (1,792 of 401k parameters moved
by ~lr = 1e-3) breaks the percentile bound; a step on stale logits, a stale W2 shadow or a
missed barrier moves most parameters by ~1e-5 .. 1e-3 and breaks the median bound.  SGD
has no normalisation: its rounding stays rounding, and its bound stays on the max."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _run(b, pst, opt, monkeypatch, sync="barrier"):
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp

    monkeypatch.setenv("JDT_MLP2_PST", pst)
    monkeypatch.setenv("JDT_MLP2_PST_SYNC", sync)
    st = init_dp(Classifier(), opt, 69, DEV)
    tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
    tr.step(b)
    eng = tr.fused
    assert eng.ahead_ok and eng.pst_ok == (pst == "1")
    tr.capture(b, steps_per_graph=7)
    tr.run_steps(b, 14)          # cold 7-step graph, then the primed one
    tr.step(b)
    tr.step(b)                   # 1-step primed graphs (one-step kernel)
    eng.forward_backward(b)      # two launches: clears the primed state
    eng.run_ahead(b, 3)          # prologue forward + one 3-step launch
    eng.run_ahead(b, 2, prologue=False)
    eng.forward_backward(b)
    tr.finalize()
    torch.cuda.synchronize()
    o = st.opt_state
    out = {"p": st.params.master.clone(), "metrics": tr.metrics.clone(), "count": int(o["count"].item()),
           "shadow": st.params.shadow.clone()}
    if "m" in o:
        out["m"], out["v"] = o["m"].clone(), o["v"].clone()
    zt = eng.ztick.cpu()
    n = 7 + 7 + 1 + 1 + 3 + 2   # run-ahead steps (one-step launches or steps of persistent launches)
    assert int(zt[0]) == 0 and int(zt[1]) == 0 and int(zt[2]) == n   # ticket re-armed, no error word, steps
    nb = 512 // 16
    assert bool((zt[32:32 * (1 + nb)].view(nb, 32)[:, 0] == 7 * n).all())   # column barriers: 7 per step
    assert bool((zt[32 * (1 + nb):].view(8, 32)[:, :28] == n).all())       # every tile once per step
    if pst == "1" and sync == "barrier":
        ws = eng.pst_ws.cpu()
        gens = 6 + 6 + 2 + 1     # grid barriers: n - 1 per persistent launch (7, 7, 3, 2)
        assert int(ws[0]) == gens and int(ws[32]) == 8 * gens
        assert bool((ws[64:320].view(8, 32)[:, 0] == 28 * gens).all())   # 224 workgroups, 28 per XCD
        assert bool((ws[320:576].view(8, 32)[:, 0] == gens).all())       # every XCD released each time
    if pst == "1" and sync == "colblk":
        ws = eng.pst_ws.cpu()
        steps = 7 + 7 + 3 + 2    # persistent steps; every one adds 7 (input chunks) per column block
        assert int(ws[1]) == steps, int(ws[1])
        assert bool((ws[32 * 18:32 * 50].view(32, 32)[:, 0] == 7 * steps).all()), ws[32 * 18:32 * 50:32]
    return out


@pytest.mark.parametrize("rows", [128, 64, 32])
def test_persistent_run_ahead_matches_per_step_launches(rows, monkeypatch):
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    g = torch.Generator().manual_seed(3)
    b = Batch(torch.randn(rows, 784, generator=g).to(DEV),
              torch.randint(0, 10, (rows,), generator=g).to(torch.int32).to(DEV))
    res = {k: _run(b, k, adamw(1e-3), monkeypatch) for k in ("0", "1")}
    assert res["0"]["count"] == res["1"]["count"] == 24
    dm = (res["0"]["metrics"] - res["1"]["metrics"]).abs()
    print(f"[pst rows {rows}] metrics {res['0']['metrics'].tolist()} |d| {dm.tolist()}")
    for k in ("p", "m", "v"):
        d = (res["0"][k] - res["1"][k]).abs().flatten().float().cpu()
        scale = float(res["0"][k].abs().max())
        ds = d.sort().values
        q50, q999 = float(ds[len(ds) // 2]), float(ds[int(0.999 * (len(ds) - 1))])
        print(f"[pst rows {rows}] {k}: max |d| {float(ds[-1]):.3e} (scale {scale:.3e}), median {q50:.3e}, "
              f"p99.9 {q999:.3e}, frac != {float((d > 0).float().mean()):.2e}")
        assert q50 <= 1e-5 * scale, (k, "median", q50)
        assert q999 <= 1e-4 * scale, (k, "p99.9", q999)
    torch.testing.assert_close(res["1"]["metrics"], res["0"]["metrics"], rtol=1e-5, atol=1e-3)
    sd = (res["0"]["shadow"].float() - res["1"]["shadow"].float()).abs()
    # the bf16 shadow may round a last-bit fp32 difference to the neighbouring bf16: one ulp
    assert float(sd.max()) <= 2.0 ** -7 * float(res["0"]["shadow"].float().abs().max())


@pytest.mark.parametrize("rows,sync", [(128, "barrier"), (64, "barrier"), (128, "colblk"), (32, "colblk")])
def test_persistent_run_ahead_deterministic_is_bitwise_equal(rows, sync, monkeypatch):
    """--deterministic (JDT_DETERMINISTIC=1) runs the benchmarked kernels too: the forward
    epilogues store per-column-block partial logits (one set per step % 3) that the next
    step's backward sums in block order, so the persistent launch and the per-step
    launches are bitwise equal -- parameters, both moments and metrics.  ``sync``: the
    between-step synchronisation of the persistent launch (grid barrier, or column-block
    completion counters: JDT_MLP2_PST_SYNC=colblk)."""
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    monkeypatch.setenv("JDT_DETERMINISTIC", "1")
    g = torch.Generator().manual_seed(5)
    b = Batch(torch.randn(rows, 784, generator=g).to(DEV),
              torch.randint(0, 10, (rows,), generator=g).to(torch.int32).to(DEV))
    res = {k: _run(b, k, adamw(1e-3), monkeypatch, sync=sync) for k in ("0", "1")}
    for k in ("p", "m", "v", "metrics", "shadow"):
        assert torch.equal(res["0"][k], res["1"][k]), (k, float((res["0"][k].float() - res["1"][k].float()).abs().max()))


def test_persistent_run_ahead_sgd(monkeypatch):
    """The fused SGD (m / v alias p, never written) through the persistent launch."""
    from jax_distributed_tuts_amd.utils.train_state import Batch, sgd

    g = torch.Generator().manual_seed(4)
    b = Batch(torch.randn(128, 784, generator=g).to(DEV),
              torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(DEV))
    res = {k: _run(b, k, sgd(0.05), monkeypatch) for k in ("0", "1")}
    d = (res["0"]["p"] - res["1"]["p"]).abs()
    assert float(d.max()) <= 1e-5 * float(res["0"]["p"].abs().max())
    torch.testing.assert_close(res["1"]["metrics"], res["0"]["metrics"], rtol=1e-5, atol=1e-3)
