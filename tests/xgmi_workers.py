"""Rank bodies for tests/test_xgmi_gpu.py: several processes share the one GPU
of the test box (gloo process group for the bootstrap), which exercises the
whole IPC path of comm/xgmi.py -- handle export/open, per-block epoch barriers
across processes, both buffer parities, graph capture -- on real hardware."""
import ctypes
import os

import torch


def _save(outdir, name, obj):
    from jax_distributed_tuts_amd.runtime import dist as D

    torch.save(obj, os.path.join(outdir, f"{name}_r{D.rank()}.pt"))


def _seq_sum(xs):
    acc = xs[0].clone()
    for x in xs[1:]:
        acc += x
    return acc


def collectives(outdir):
    from jax_distributed_tuts_amd.comm.xgmi import XgmiComm, part_len
    from jax_distributed_tuts_amd.ops import kernels as K
    from jax_distributed_tuts_amd.runtime import dist as D

    r, W, dev = D.rank(), D.world_size(), D.device()
    mesh = D.Mesh({"data": W})
    comm = XgmiComm(mesh.group("data"), r, W, 1 << 21, dev, timeout_s=20.0)
    res = {"ok": comm.ok}
    if not comm.ok:
        _save(outdir, "xg", res)
        return
    # all-reduce: bit-exact vs the rank-ordered fp32 sum, odd sizes, repeated calls
    ar = {}
    for n in (1, 3, 4, 1000, 407168, 1_999_999):
        xs = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * q + n % 997)) for q in range(W)]
        y = xs[r].to(dev)
        comm.all_reduce_(y)
        ar[n] = bool(torch.equal(y.cpu(), _seq_sum(xs)))
    # small sizes take the one-shot kernel (<= 256 KiB); the same sizes forced through
    # the two-shot kernel, interleaved with one-shot calls (shared epochs / parities)
    for n in (1000, 50_000):
        xs = [torch.randn(n, generator=torch.Generator().manual_seed(77 * q + n)) for q in range(W)]
        for forced in (0, 256 * 1024, 0):
            XgmiComm.set_oneshot_bytes(forced)
            y = xs[r].to(dev)
            comm.all_reduce_(y)
            ar[f"{'2shot' if forced == 0 else '1shot'}_{n}_{len(ar)}"] = bool(torch.equal(y.cpu(), _seq_sum(xs)))
    XgmiComm.set_oneshot_bytes(256 * 1024)
    res["ar"] = ar
    # per-size transport choice: one-shot / two-shot / RCCL timed at the
    # DP bucket, threshold set to the measured crossover; all-reduce still exact after it
    from jax_distributed_tuts_amd.comm.xgmi import calibrate
    from jax_distributed_tuts_amd.ops import _lib as _L

    cal = calibrate(comm, [407_168], iters=5)
    res["cal_rccl"] = cal["rccl"]
    res["cal_rows"] = len(cal["table"])
    res["cal_threshold_ok"] = cal["oneshot_threshold_bytes"] in [0] + [row["bytes"] for row in cal["table"]]
    res["cal_threshold_set"] = int(_L.lib().jdt_xgmi_oneshot_bytes()) == cal["oneshot_threshold_bytes"]
    res["cal_has_bucket"] = any(row["trainer_size"] for row in cal["table"])
    xs = [torch.randn(5000, generator=torch.Generator().manual_seed(9 + q)) for q in range(W)]
    y = xs[r].to(dev)
    comm.all_reduce_(y)
    res["ar_after_cal"] = bool(torch.equal(y.cpu(), _seq_sum(xs)))
    XgmiComm.set_oneshot_bytes(256 * 1024)
    # the production geometry: create_for sizes the context to the trainer's bucket (the DP
    # tutorial's 407,050 grads + 4 metric slots) and must time exactly that size, then pick
    # the transport from that row
    from jax_distributed_tuts_amd.comm import xgmi as XM

    prod = XM.create_for(mesh, "data", 407_054, dev, "xgmi")
    cal2 = XM.LAST_CALIBRATION or {}
    rows = [row for row in cal2.get("table", []) if row["trainer_size"]]
    res["prod_trainer_row"] = (prod is not None and len(rows) == 1 and rows[0]["bytes"] == 4 * 407_054
                               and cal2.get("transport") == "xgmi" and rows[0]["xgmi_twoshot_us"] > 0)
    if prod is not None:
        prod.close()
    XgmiComm.set_oneshot_bytes(256 * 1024)
    # fused all-reduce + AdamW + metrics fold == sum, then the standalone AdamW kernel
    npar, total = 4096, 4096 + 64
    g = torch.Generator().manual_seed(7)
    p0 = torch.randn(npar, generator=g)
    m0 = torch.randn(npar, generator=g) * 1e-2
    v0 = torch.rand(npar, generator=g) * 1e-2
    run0 = torch.tensor([1.0, 2.0, 3.0, 4.0])
    p, m, v = p0.to(dev), m0.to(dev), v0.to(dev)
    sh = torch.empty(npar, dtype=torch.bfloat16, device=dev)
    run = run0.to(dev)
    step = torch.tensor([5], dtype=torch.int32, device=dev)
    ticket = torch.zeros(1, dtype=torch.int32, device=dev)
    pr, mr, vr = p0.to(dev), m0.to(dev), v0.to(dev)
    shr = torch.empty_like(sh)
    stepr = torch.tensor([5], dtype=torch.int32, device=dev)
    ticketr = torch.zeros(1, dtype=torch.int32, device=dev)
    runr = run0.clone()
    fused = {"p": True, "m": True, "v": True, "shadow": True, "running": True, "step": True, "zero": True}
    for it in range(3):
        gs = [torch.randn(total, generator=torch.Generator().manual_seed(50 + 10 * it + q)) for q in range(W)]
        gsum = _seq_sum(gs)
        gr = gs[r].to(dev)
        comm.all_reduce_adamw_(gr, p=p, m=m, v=v, shadow=sh, n_params=npar, running=run, n_metrics=4, lr=1e-3,
                               b1=0.9, b2=0.999, eps=1e-8, wd=1e-4, grad_scale=0.25, step=step, ticket=ticket)
        K.adamw_step(pr, gsum[:npar].to(dev), mr, vr, shr, lr=1e-3, grad_scale=0.25, step=stepr, ticket=ticketr)
        runr += gsum[npar:npar + 4]
        torch.cuda.synchronize()
        # the two AdamW kernels may contract FMAs differently: 1-ulp differences allowed,
        # the bf16 shadow must be exactly the rounding of this kernel's own master copy
        fused["p"] &= bool(torch.allclose(p, pr, rtol=1e-6, atol=1e-7))
        fused["m"] &= bool(torch.allclose(m, mr, rtol=1e-5, atol=1e-8))
        fused["v"] &= bool(torch.allclose(v, vr, rtol=1e-5, atol=1e-9))
        fused["shadow"] &= bool(torch.equal(sh, p.to(torch.bfloat16)))
        fused["running"] &= bool(torch.allclose(run.cpu(), runr, rtol=1e-6, atol=1e-6))
        fused["step"] &= int(step.item()) == 6 + it and int(ticket.item()) == 0
        fused["zero"] &= bool((gr == 0).all())
    # per-bucket calls of one step (parallel/pipeline._overlapped_sync): the first holds
    # the step counter (advance=False), the last advances it and folds the metrics --
    # equal to one call over the whole bucket
    gs = [torch.randn(total, generator=torch.Generator().manual_seed(90 + q)) for q in range(W)]
    outs = []
    for split in (False, True):
        pa, ma, va = p0.to(dev), m0.to(dev), v0.to(dev)
        sa, ra = torch.empty_like(sh), run0.to(dev)
        sta, tka = torch.tensor([5], dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int32, device=dev)
        ga = gs[r].to(dev)
        kw = dict(lr=1e-3, b1=0.9, b2=0.999, eps=1e-8, wd=1e-4, grad_scale=0.25, step=sta, ticket=tka)
        if split:
            c = 2048
            comm.all_reduce_adamw_(ga[:c], p=pa[:c], m=ma[:c], v=va[:c], shadow=sa[:c], n_params=c, running=None,
                                   n_metrics=0, advance=False, **kw)
            comm.all_reduce_adamw_(ga[c:], p=pa[c:], m=ma[c:], v=va[c:], shadow=sa[c:], n_params=npar - c,
                                   running=ra, n_metrics=4, **kw)
        else:
            comm.all_reduce_adamw_(ga, p=pa, m=ma, v=va, shadow=sa, n_params=npar, running=ra, n_metrics=4, **kw)
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in (pa, ma, va, sa, ra, sta, tka, ga)])
    res["bucketed"] = all(torch.equal(x, y) for x, y in zip(*outs)) and int(outs[1][5].item()) == 6
    res["fused_detail"] = fused
    fused_ok = all(fused.values())
    res["fused"] = fused_ok
    # reduce-scatter / all-gather with a caller part size
    n = 10_001
    part = part_len(n, W)
    fulls = [torch.randn(n, generator=torch.Generator().manual_seed(300 + q)) for q in range(W)]
    out = torch.full((part,), -1.0, device=dev)
    comm.reduce_scatter(fulls[r].to(dev), out, part)
    lo, hi = r * part, min(n, (r + 1) * part)
    res["rs"] = bool(torch.equal(out[: hi - lo].cpu(), _seq_sum(fulls)[lo:hi]))
    shards = [torch.randn(part, generator=torch.Generator().manual_seed(400 + q)) for q in range(W)]
    outg = torch.empty(n, device=dev)
    comm.all_gather(shards[r].to(dev), outg, part)
    res["ag"] = bool(torch.equal(outg.cpu(), torch.cat(shards)[:n]))
    # hipGraph: two all-reduces captured once, replayed three times
    base = (torch.arange(50_000) % 13).float()
    x = (base + r).to(dev)
    gph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gph):
        comm.all_reduce_(x)
        comm.all_reduce_(x)
    want = (base * W + W * (W - 1) / 2) * W
    gok = True
    for _ in range(3):
        x.copy_((base + r).to(dev))
        gph.replay()
        torch.cuda.synchronize()
        gok &= bool(torch.equal(x.cpu(), want))
    res["graph"] = gok
    res["err"] = comm.error()
    _save(outdir, "xg", res)
    comm.close()


def dp_xgmi(outdir, steps_eager=2, steps_graph=6, dp_ahead="1", num_layers=2, width=(784, 512), dp_pst="1", tag=""):
    """DP over the xGMI fused all-reduce+AdamW kernel (dropout off), fused step
    kernels, eager steps then multi-step graph replays.  ``dp_ahead`` = JDT_DP_AHEAD:
    "1" lets the step be one run-ahead launch with the in-kernel tile exchange where
    every rank's grid fits on the shared GPU, "0" keeps the three-launch step.
    ``width`` = (input size, hidden size) of the classifier.  ``dp_pst`` = JDT_DP_PST: "1"
    lets a multi-step replay of the one-launch step be ONE persistent launch per rank (the
    exchange inside every step, mlp2_pst_kernel TX), "0" one run-ahead launch per step."""
    os.environ["JDT_DP_AHEAD"] = dp_ahead
    os.environ["JDT_DP_PST"] = dp_pst
    os.environ["JDT_DP_DEEP_TX"] = dp_ahead   # the deep engine's exchange path is opt-in: test it
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp, shard_batch
    from jax_distributed_tuts_amd.runtime import dist as D
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    dev = D.device()
    cfg = dp_config()
    cfg.data.input_size = width[0]
    mesh = D.Mesh({"data": D.world_size()})
    st = init_dp(Classifier(input_size=width[0], hidden_size=width[1], num_layers=num_layers, dropout_rate=0.0),
                 adamw(1e-3), 69, dev, None)  # same seed
    b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    tr = DataParallelTrainer(st, mesh, DPConfig(4, "kernel", comm="xgmi"))
    assert tr.xg is not None and tr.fused is None
    for _ in range(steps_eager):
        tr.step(b)
    tr.capture(b, steps_per_graph=3)
    tr.run_steps(b, steps_graph)
    torch.cuda.synchronize()
    tr.finalize()
    _save(outdir, "dpx" + tag, {"master": st.params.master.cpu(), "metrics": tr.metrics.cpu(),
                                "comm": tr.comm_backend, "fused": tr.fused is not None,
                                "step": int(st.opt_state["count"].item()), "one_launch": bool(tr.one_launch),
                                "m": st.opt_state["m"].cpu(), "v": st.opt_state["v"].cpu(),
                                "pst": bool(getattr(tr.fused, "pst_ok", False))})


def fsdp_xgmi(outdir, fused=True, steps=3, num_layers=2, eps=1e-8, deep_fx="0", hidden=512, pst="1", tag=""):
    """FSDP (dropout off) with the segmented xGMI gather / reduce-scatter; every rank
    saves its local shard + the partition table for reassembly in the parent.
    num_layers=4: the square 512 x 512 hidden weights are sharded along dim 1 (the
    reference rule) and move as 2-D column-block segments.  deep_fx = JDT_FSDP_DEEP_FX."""
    import os

    os.environ["JDT_FSDP_DEEP_FX"] = deep_fx
    os.environ["JDT_FSDP_PST"] = pst   # 1: multi-step replays of the one-launch step as ONE persistent launch
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.runtime import dist as D
    from jax_distributed_tuts_amd.utils.config import fsdp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw

    dev = D.device()
    cfg = fsdp_config()
    mesh = D.Mesh({"data": D.world_size()})
    st = init_fsdp(Classifier(hidden_size=hidden, num_layers=num_layers, dropout_rate=0.0), adamw(1e-3, eps=eps), 69,
                   dev, mesh, "data", 16)
    b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=fused,
                                          comm="xgmi"))
    tr.step(b)
    assert tr.capturable
    tr.capture(b, steps_per_graph=2)  # the rest of the steps replay one hipGraph (collectives are kernels)
    tr.run_steps(b, steps - 1)
    torch.cuda.synchronize()
    tr.finalize()
    sp = st.extra["sharded"]
    o = st.opt_state
    _save(outdir, f"fsx{num_layers}{tag}", {"local": {n: sp.local.p(n).cpu() for n in sp.part},
                          "m": o["m"][:sp.local.numel].cpu(), "v": o["v"][:sp.local.numel].cpu(),
                          "pst": bool(getattr(getattr(tr, "fused", None), "pst_ok", False)),
                          "offsets": {n: (o_, int(torch.Size(s_).numel())) for n, (o_, s_) in sp.local.offsets.items()},
                          "dims": {n: sp.part[n].shard_dim for n in sp.part},
                          "metrics": tr.metrics.cpu(), "comm": tr.comm_backend, "xg_names": list(sp._xg_names),
                          "fused_comm": getattr(tr, "_plan", None) is not None or tr.one_launch,
                          "one_launch": bool(tr.one_launch)})


def pp_xgmi(outdir, dp, n_hidden=3, steps=4, pp_kernel="1", dropout=0.0, tag="", n_mb=4):
    """GPipe with the xGMI inbox hand-off (+ the fused xGMI all-reduce on the data axis
    when dp > 1): one eager step, then multi-step graph replays.  ``pp_kernel`` =
    JDT_PP_KERNEL: "1" lets a pipeline of one layer per stage run each stage's step as
    one persistent launch (parallel/pp_kernel.py), "0" keeps the per-tick launches."""
    os.environ["JDT_PP_KERNEL"] = pp_kernel
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.runtime import dist as D
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch

    dev = D.device()
    cfg = dp_config()
    mesh = D.Mesh({"data": dp, "pipe": D.world_size() // dp})
    tr = build_mlp_pipeline(cfg, mesh, dev, n_hidden_layers=n_hidden, dropout_rate=dropout, num_microbatches=n_mb,
                            comm="xgmi")
    b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    tr.step(b)
    assert tr.capturable and (tr.p2p is not None or tr.pp_kernel is not None)
    tr.capture(b, steps_per_graph=2)
    tr.run_steps(b, steps - 1)
    torch.cuda.synchronize()
    tr.finalize()
    _save(outdir, f"ppx{dp}{tag}", {"params": {k: v.cpu() for k, v in tr.state.params.state_dict().items()},
                                    "metrics": tr.gather_metrics().cpu(), "comm": tr.comm_backend,
                                    "count": int(tr.state.step_tensor.item()),
                                    "pp_kernel": tr.pp_kernel is not None})


def pp_restore(outdir, n_hidden, pp_kernel="1", dropout=0.1, tag=""):
    """GPipe over the inboxes: 2 steps, checkpoint, 3 more steps (the hand-off flags move
    past the checkpoint's epochs), restore, then 1 eager step + a 2-step graph replay.
    With the stage kernel the restore must rebuild its engine (parallel/pipeline.py
    invalidate): stale flags would let every in-kernel wait pass at once."""
    os.environ["JDT_PP_KERNEL"] = pp_kernel
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.runtime import dist as D
    from jax_distributed_tuts_amd.utils import checkpoint as CK
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch

    dev = D.device()
    cfg = dp_config()
    mesh = D.Mesh({"data": 1, "pipe": D.world_size()})
    tr = build_mlp_pipeline(cfg, mesh, dev, n_hidden_layers=n_hidden, dropout_rate=dropout, num_microbatches=4,
                            comm="xgmi")
    b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    for _ in range(2):
        tr.step(b)
    torch.cuda.synchronize()
    ck = os.path.join(outdir, f"ck{tag}")
    CK.save(tr.state, ck, tr.metrics)
    D.barrier()
    for _ in range(3):
        tr.step(b)
    torch.cuda.synchronize()
    D.barrier()
    CK.restore(tr.state, ck, tr.metrics)
    tr.step(b)
    tr.capture(b, steps_per_graph=2)
    tr.run_steps(b, 2)
    torch.cuda.synchronize()
    tr.finalize()
    _save(outdir, f"ppr{tag}", {"params": {k: v.cpu() for k, v in tr.state.params.state_dict().items()},
                                "metrics": tr.gather_metrics().cpu(),
                                "count": int(tr.state.step_tensor.item()),
                                "pp_kernel": tr.pp_kernel is not None})


def p2p_roundtrip(outdir):
    """Raw XgmiP2P: ring sends through every slot, eager and graph-replayed epochs."""
    from jax_distributed_tuts_amd.comm.p2p import XgmiP2P
    from jax_distributed_tuts_amd.runtime import dist as D

    r, W, dev = D.rank(), D.world_size(), D.device()
    mesh = D.Mesh({"pipe": W})
    n_slots = 6
    c = XgmiP2P(mesh.group("pipe"), r, W, 70_000, n_slots, dev, timeout_s=20.0)
    res = {"ok": c.ok}
    if c.ok:
        ep = torch.zeros(1, dtype=torch.int32, device=dev)
        sizes = [16, 4096, 65_536, 70_000 // 16 * 16]
        xs = [torch.arange(n // 4, device=dev, dtype=torch.float32) * (r + 1) + k for k, n in enumerate(sizes)]
        outs = [torch.empty_like(x) for x in xs]

        def body():
            for k, x in enumerate(xs):
                c.send(x, (r + 1) % W, k, ep)
            for k, o in enumerate(outs):
                c.recv(o, k, ep)
            ep.add_(1)

        body()
        torch.cuda.synchronize()
        prev = (r - 1) % W
        good = all(torch.equal(o, torch.arange(o.numel(), device=dev, dtype=torch.float32) * (prev + 1) + k)
                   for k, o in enumerate(outs))
        D.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        for it in range(3):
            for k, x in enumerate(xs):
                x.add_(1)
            torch.cuda.synchronize()
            D.barrier()  # every rank has read the previous epoch
            g.replay()
            torch.cuda.synchronize()
            good &= all(torch.equal(o, torch.arange(o.numel(), device=dev, dtype=torch.float32) * (prev + 1) + k
                                    + it + 1) for k, o in enumerate(outs))
        res["data"] = good
        res["epoch"] = int(ep.item())
        res["err"] = c.error()
        c.close()
    _save(outdir, "p2p", res)


def lm_pp_xgmi(outdir, dp, steps=3, n_layers=2):
    """Transformer LM (small config) over a (data=dp, pipe=W/dp) mesh with the xGMI
    inbox hand-off and the fused data-axis all-reduce; eager step, then graphs."""
    from jax_distributed_tuts_amd.models.transformer import TransformerConfig
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline, lm_batch
    from jax_distributed_tuts_amd.runtime import dist as D
    from jax_distributed_tuts_amd.utils.train_state import Batch

    dev = D.device()
    cfg = TransformerConfig(vocab_size=512, d_model=128, n_heads=2, d_ff=256, seq_len=64, n_layers=n_layers)
    mesh = D.Mesh({"data": dp, "pipe": D.world_size() // dp})
    tr, _ = build_lm_pipeline(mesh, dev, cfg, num_microbatches=2, comm="xgmi")
    tr.cfg.overlap_data_sync = "1"   # "auto" keeps it off with ranks sharing the GPU; test the path
    b = shard_batch(lm_batch(cfg, global_batch=8, seed=1), mesh, "data")
    b = Batch(b.inputs.to(dev), b.labels.to(dev))
    tr.step(b)
    assert tr.capturable and tr.p2p is not None
    tr.capture(b, steps_per_graph=2)
    tr.run_steps(b, steps - 1)
    torch.cuda.synchronize()
    tr.finalize()
    _save(outdir, f"lmx{dp}", {"params": {k: v.cpu() for k, v in tr.state.params.state_dict().items()},
                               "metrics": tr.gather_metrics().cpu(), "comm": tr.comm_backend,
                               "buckets": len(getattr(tr, "_buckets", None) or [])})


def tile_exchange(outdir):
    """The one-launch DP step's tile exchange (comm/tile_exchange.py) at W ranks: buffers
    exported / mapped, the start-up self-test (every payload position of 64 tiles summed
    over the W ranks, bit-exact) passes, flags cleared."""
    from jax_distributed_tuts_amd.comm.tile_exchange import TileExchange
    from jax_distributed_tuts_amd.runtime import dist as D

    r, W, dev = D.rank(), D.world_size(), D.device()
    mesh = D.Mesh({"data": W})
    tx = TileExchange(mesh.group("data"), r, W, 224, dev, timeout_s=20.0)
    res = {"ok": tx.ok, "selftest": tx.selftest, "args": tx.args_ptr != 0}
    tx.close()
    _save(outdir, "tx", res)


def fault_timeout(outdir):
    """Fault injection: rank 1 never joins the collective / never sends.  Rank 0's
    in-kernel waits must time out into the error flag (no hung GPU), for both
    the xGMI all-reduce and the pipeline inbox receive."""
    from jax_distributed_tuts_amd.comm.p2p import XgmiP2P
    from jax_distributed_tuts_amd.comm.xgmi import XgmiComm
    from jax_distributed_tuts_amd.runtime import dist as D

    r, W, dev = D.rank(), D.world_size(), D.device()
    mesh = D.Mesh({"data": W})
    comm = XgmiComm(mesh.group("data"), r, W, 1 << 16, dev, timeout_s=1.0)
    p2p = XgmiP2P(mesh.group("data"), r, W, 4096, 2, dev, timeout_s=1.0)
    res = {"ok": comm.ok and p2p.ok}
    D.barrier()
    if r == 0:
        x = torch.ones(1000, device=dev)
        comm.all_reduce_(x)                      # peer absent: both barriers time out
        res["ar_err"] = comm.error()
        out = torch.empty(256, device=dev)
        ep = torch.zeros(1, dtype=torch.int32, device=dev)
        p2p.recv(out, 0, ep)                     # nobody sends
        res["p2p_err"] = p2p.error()
    D.barrier()
    _save(outdir, "fault", res)
    comm.close()
    p2p.close()


def grad_probe_xgmi(outdir, kind, dp=1, capture=True, n_hidden=3):
    """One step (dropout off) of a strategy over the xGMI kernels with a
    scale-revealing optimizer -- plain SGD lr 1, or (``dp_adam_eps``) the fused
    xGMI all-reduce + AdamW kernel with eps = 10 -- saving params before / after
    (tests/test_grad_scale_gpu.py)."""
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp, shard_batch
    from jax_distributed_tuts_amd.runtime import dist as D
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch, adamw, sgd

    dev = D.device()
    cfg = dp_config()

    def cpu(d):
        return {k: v.detach().float().cpu().clone() for k, v in d.items()}

    extra = {}
    if kind in ("dp_sgd", "dp_adam_eps", "dp4_adam_eps"):
        os.environ["JDT_DP_DEEP_TX"] = "1"   # dp4: the deep engine's (opt-in) exchange path where it fits
        mesh = D.Mesh({"data": D.world_size()})
        tx = sgd(1.0) if kind == "dp_sgd" else adamw(1.0, eps=10.0, weight_decay=0.0)
        st = init_dp(Classifier(num_layers=4 if kind == "dp4_adam_eps" else 2, dropout_rate=0.0), tx, 69, dev, None)
        b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
        tr = DataParallelTrainer(st, mesh, DPConfig(4, "kernel", comm="xgmi"))
        before = cpu(st.params.state_dict())
        tr.step(Batch(b.inputs.to(dev), b.labels.to(dev)))
        tr.finalize()
        after = cpu(st.params.state_dict())
        comm = tr.comm_backend
    elif kind == "fsdp_sgd":
        from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp

        mesh = D.Mesh({"data": D.world_size()})
        st = init_fsdp(Classifier(dropout_rate=0.0), sgd(1.0), 69, dev, mesh, "data", 16)
        b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
        tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=True,
                                              comm="xgmi"))
        before = cpu(tr.full_params())
        tr.step(Batch(b.inputs.to(dev), b.labels.to(dev)))
        tr.finalize()
        after = cpu(tr.full_params())
        comm = tr.comm_backend
    elif kind == "fsdp_loop_sgd":
        # the reference's per-minibatch gather / reduce-scatter schedule on the fused md
        # kernels (FSDPConfig.fused_loop), the probed step replayed from a hipGraph
        from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp

        mesh = D.Mesh({"data": D.world_size()})
        st = init_fsdp(Classifier(dropout_rate=0.0), sgd(1.0), 69, dev, mesh, "data", 16)
        b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
        b = Batch(b.inputs.to(dev), b.labels.to(dev))
        tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data", gather_once=False, scatter_once=False,
                                              fused_kernels=False, comm="xgmi"))
        tr.step(b)   # eager: builds the loop engine
        assert tr._loop_engine is not None and tr.capturable
        torch.cuda.synchronize()
        before = cpu(tr.full_params())
        if capture:
            tr.capture(b)
        tr.step(b)   # graph replay (or a second eager step)
        tr.finalize()
        after = cpu(tr.full_params())
        comm = tr.comm_backend
    elif kind == "fsdp4_adam_eps":
        # the deep FSDP step with every hidden layer's backward sending its partials to the
        # shard owners (md_bwd FX, JDT_FSDP_DEEP_FX=1; at 8 shared ranks the grids do not
        # fit: the step collective form)
        from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp

        os.environ["JDT_FSDP_DEEP_FX"] = "1"
        mesh = D.Mesh({"data": D.world_size()})
        st = init_fsdp(Classifier(num_layers=4, dropout_rate=0.0), adamw(1.0, eps=10.0, weight_decay=0.0), 69, dev,
                       mesh, "data", 16)
        b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
        tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True, fused_kernels=True,
                                              comm="xgmi"))
        before = cpu(tr.full_params())
        tr.step(Batch(b.inputs.to(dev), b.labels.to(dev)))
        tr.finalize()
        after = cpu(tr.full_params())
        comm = tr.comm_backend
        extra["one_launch"] = bool(tr.one_launch)
    elif kind in ("pp_sgd", "pp_adam_eps"):
        from pipeline_parallel import build_mlp_pipeline

        mesh = D.Mesh({"data": dp, "pipe": D.world_size() // dp})
        # pp_adam_eps with one layer per stage: the in-kernel GPipe stage step (AdamW only)
        tx = sgd(1.0) if kind == "pp_sgd" else adamw(1.0, eps=10.0, weight_decay=0.0)
        tr = build_mlp_pipeline(cfg, mesh, dev, n_hidden_layers=n_hidden, dropout_rate=0.0, num_microbatches=4,
                                comm="xgmi", tx=tx)
        b = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
        before = cpu(tr.state.params.state_dict())
        tr.step(Batch(b.inputs.to(dev), b.labels.to(dev)))
        tr.finalize()
        after = cpu(tr.state.params.state_dict())
        comm = tr.comm_backend
        extra["pp_kernel"] = getattr(tr, "pp_kernel", None) is not None
    else:
        raise ValueError(kind)
    torch.cuda.synchronize()
    _save(outdir, f"gpx_{kind}", {"before": before, "after": after, "comm": comm, **extra})


def ipc_churn(outdir, iters=6, pool="0"):
    """Comm contexts built, used and torn down (two-phase) in a loop with torch tensors
    allocated between them (canaries), the exported-buffer pool OFF: every self-test must
    pass and no canary may change (a write through a stale peer mapping would)."""
    os.environ["JDT_IPC_POOL"] = pool
    import torch.distributed as dist

    from jax_distributed_tuts_amd.comm import xgmi as X
    from jax_distributed_tuts_amd.ops import _lib
    from jax_distributed_tuts_amd.runtime import dist as D

    dev = D.device()
    rank, world = D.rank(), D.world_size()
    X.size_grids_for_sharing(dev)
    fails = bad = 0
    held = []
    for it in range(iters):
        c = X.XgmiComm(dist.group.WORLD, rank, world, 408_576, dev, timeout_s=D.spin_timeout_s(30.0))
        fails += int(not c.ok)
        if c.ok:
            x = torch.ones(407_054, device=dev) * (rank + 1)
            for _ in range(20):
                c.all_reduce_(x)
        torch.cuda.synchronize(dev)
        bad += sum(int(not bool((t == v).all())) for t, v in held)
        D.quiesce(dev)
        c.close()
        held = []
        for k, n in enumerate((1 << 17, 1 << 19, 1 << 21)):
            v = float(100 * it + 10 * k + rank + 1)
            held.append((torch.full((n,), v, device=dev), v))
        D.barrier()
    st = (ctypes.c_long * 3)()
    _lib.lib().jdt_ipc_pool_stats(st)
    _save(outdir, "churn", {"fails": fails, "bad": bad, "pool_buffers": int(st[0]), "pool_in_use": int(st[2])})
