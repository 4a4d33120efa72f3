"""Worker bodies for the multi-process gloo tests (importable by spawned children)."""
import os

import torch

from jax_distributed_tuts_amd.comm import collectives as C
from jax_distributed_tuts_amd.runtime import dist as D
from jax_distributed_tuts_amd.runtime.dist import Mesh


def _save(out_dir, name, obj):
    torch.save(obj, os.path.join(out_dir, f"{name}_r{D.rank()}.pt"))


def collectives(out_dir):
    ws, r = D.world_size(), D.rank()
    mesh = Mesh({"data": ws})
    x = torch.arange(8, dtype=torch.float32) + 100 * r
    res = {}
    res["psum"] = C.psum_(x.clone(), mesh, "data")
    res["pmean"] = C.pmean_(x.clone(), mesh, "data")
    res["ag0"] = C.all_gather(x.view(2, 4), mesh, "data", dim=0)
    res["ag1"] = C.all_gather(x.view(2, 4), mesh, "data", dim=1)
    res["rs"] = C.psum_scatter(torch.arange(4 * ws, dtype=torch.float32).view(2 * ws, 2) * (r + 1), mesh, "data")
    res["ring"] = C.ppermute(x, mesh, "data", [(i, (i + 1) % ws) for i in range(ws)])
    res["idx"] = C.axis_index(mesh, "data")
    _save(out_dir, "coll", res)


def mesh2d(out_dir):
    mesh = Mesh({"data": 2, "pipe": D.world_size() // 2})
    x = torch.tensor([float(D.rank())])
    res = {"coords": mesh.coords, "data_sum": C.psum_(x.clone(), mesh, "data"),
           "pipe_sum": C.psum_(x.clone(), mesh, "pipe"), "pipe_ranks": mesh.group_ranks("pipe"),
           "data_ranks": mesh.group_ranks("data")}
    _save(out_dir, "mesh", res)


def gather_mean_grad(out_dir):
    from jax_distributed_tuts_amd.parallel.fsdp import gather_arr_mean_grads

    ws, r = D.world_size(), D.rank()
    mesh = Mesh({"data": ws})
    shard = (torch.arange(6, dtype=torch.float32).view(3, 2) + 10 * r).requires_grad_()
    full = gather_arr_mean_grads(shard, mesh, "data", 0)
    w = torch.arange(full.numel(), dtype=torch.float32).view_as(full) * (r + 1)
    (full * w).sum().backward()
    _save(out_dir, "gmg", {"full": full.detach(), "grad": shard.grad})


def dp_vs_single(out_dir, accum):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp, shard_batch
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import adamw

    cfg = dp_config()
    mesh = Mesh({"data": D.world_size()})
    model = Classifier(dropout_rate=0.0)
    st = init_dp(model, adamw(1e-3), 69, "cpu", mesh)
    batch = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    tr = DataParallelTrainer(st, mesh, DPConfig(4, accum))
    for _ in range(3):
        tr.step(batch)
    _save(out_dir, f"dp_{accum}", {"params": st.params.state_dict(), "metrics": tr.metrics.clone()})


def fsdp_run(out_dir, gather_once):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import adamw

    cfg = dp_config()
    mesh = Mesh({"data": D.world_size()})
    model = Classifier(dropout_rate=0.0)
    st = init_fsdp(model, adamw(1e-3), 69, "cpu", mesh, "data", 16)
    batch = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data", gather_once=gather_once, scatter_once=gather_once))
    for _ in range(3):
        tr.step(batch)
    _save(out_dir, f"fsdp_{int(gather_once)}", {"params": tr.full_params(), "metrics": tr.metrics.clone()})


def sharded_module(out_dir):
    from jax_distributed_tuts_amd.parallel.fsdp import shard_module_params, sync_gradients

    ws = D.world_size()
    mesh = Mesh({"data": ws})
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(16, 8), torch.nn.Tanh(), torch.nn.Linear(8, 4))
    ref = {n: p.detach().clone() for n, p in net.named_parameters()}
    sm = shard_module_params(net, mesh, "data", min_weight_size=4)
    g = torch.Generator().manual_seed(D.rank())
    x = torch.randn(5, 16, generator=g)
    out = sm(x)
    out.square().mean().backward()
    grads = sync_gradients(sm.partitioned_grads(), mesh, ["data"])
    _save(out_dir, "sm", {"ref": ref, "x": x, "out": out.detach(),
                          "grads": {k: (v.value if hasattr(v, "value") else v) for k, v in grads.items()},
                          "meta": sm.meta})


def pp_run(out_dir, dp, n_hidden=3, n_mb=4, steps=3):
    from data_paral import synthetic_batch
    from pipeline_parallel import build_mlp_pipeline
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.utils.config import dp_config

    cfg = dp_config()
    mesh = Mesh({"data": dp, "pipe": D.world_size() // dp})
    tr = build_mlp_pipeline(cfg, mesh, "cpu", n_hidden_layers=n_hidden, dropout_rate=0.0, num_microbatches=n_mb)
    batch = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    for _ in range(steps):
        tr.step(batch)
    _save(out_dir, f"pp_dp{dp}", {"params": tr.state.params.state_dict(), "metrics": tr.gather_metrics()})


def replication(out_dir):
    from jax_distributed_tuts_amd.utils.debug import ReplicationError, check_replicated

    mesh = Mesh({"data": D.world_size()})
    same = {"w": torch.arange(10.0)}
    check_replicated(same, mesh, "data")
    diff = {"w": torch.arange(10.0) + (D.rank() == 1)}
    try:
        check_replicated(diff, mesh, "data")
        res = "no-error"
    except ReplicationError as e:
        res = str(e)
    _save(out_dir, "rep", {"res": res})


def ckpt(out_dir):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import shard_batch
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils import checkpoint
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import adamw

    cfg = dp_config()
    mesh = Mesh({"data": D.world_size()})
    batch = shard_batch(synthetic_batch(cfg, 70), mesh, "data")

    def make():
        st = init_fsdp(Classifier(dropout_rate=0.0), adamw(1e-3), 69, "cpu", mesh, "data", 16)
        return st, FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data"))

    st, tr = make()
    for _ in range(2):
        tr.step(batch)
    checkpoint.save(st, os.path.join(out_dir, "ck"), tr.metrics)
    tr.step(batch)
    ref = tr.full_params()
    st2, tr2 = make()
    checkpoint.restore(st2, os.path.join(out_dir, "ck"), tr2.metrics)
    tr2.step(batch)
    _save(out_dir, "ck", {"ref": ref, "got": tr2.full_params(), "step": st2.step,
                          "count": int(st2.opt_state["count"])})


def dp_overlap(out_dir, overlap, bucket_mb):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp, shard_batch
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import adamw

    cfg = dp_config()
    mesh = Mesh({"data": D.world_size()})
    st = init_dp(Classifier(dropout_rate=0.0, num_layers=4), adamw(1e-3), 69, "cpu", mesh)
    batch = shard_batch(synthetic_batch(cfg, 70), mesh, "data")
    tr = DataParallelTrainer(st, mesh, DPConfig(4, "loop", overlap=overlap, bucket_mb=bucket_mb))
    nb = len(tr.buckets.ranges) if tr.buckets is not None else 0
    for _ in range(2):
        tr.step(batch)
    _save(out_dir, f"ov{int(overlap)}", {"params": st.params.state_dict(), "metrics": tr.metrics.clone(), "nb": nb})


# ----------------------------------------------------------------------------- gradient-scale probes
def _clone(d):
    return {k: v.detach().clone() for k, v in d.items()}


LM_PROBE_CFG = dict(vocab_size=64, d_model=64, n_heads=4, d_ff=128, seq_len=16, n_layers=4)


def grad_probe(out_dir, kind, accum="loop", gather_once=False, dp=1, n_hidden=3, num_layers=2, n_mb=4):
    """ONE plain-SGD (lr 1) step of a strategy, dropout off; saves the parameters
    before and after, so the test reads the applied gradient p0 - p1 exactly
    (tests/oracle.py)."""
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.ops import kernels as K
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp, shard_batch
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import sgd

    cfg = dp_config()
    batch_full = synthetic_batch(cfg, 70)
    if kind == "dp_drop4":
        # throwaway fault: rank 0's first minibatch loses its first 4-row group
        orig, calls = K.softmax_xent, [0]

        def dropped(logits, labels, *, dlogits=None, **kw):
            calls[0] += 1
            if D.rank() != 0 or calls[0] != 1:
                return orig(logits, labels, dlogits=dlogits, **kw)
            dlogits[:4].zero_()
            return orig(logits[4:], labels[4:], dlogits=dlogits[4:], **kw)

        K.softmax_xent = dropped
        kind = "dp"
    if kind in ("dp", "dp_no_inv_n"):
        mesh = Mesh({"data": D.world_size()})
        st = init_dp(Classifier(dropout_rate=0.0, num_layers=num_layers), sgd(1.0), 69, "cpu", mesh)
        cls = DataParallelTrainer
        if kind == "dp_no_inv_n":
            class _NoInvN(DataParallelTrainer):  # deliberately drops the 1/N of pmean
                def update_noncounting(self):
                    P = self.state.params
                    self.state.tx.update(P, self.state.opt_state, 1.0 / self.cfg.num_minibatches)
                    K.metrics_fold_(self.metrics, P.metrics_slot)
            cls = _NoInvN
        tr = cls(st, mesh, DPConfig(4, accum))
        before = _clone(st.params.state_dict())
        tr.step(shard_batch(batch_full, mesh, "data"))
        after = _clone(st.params.state_dict())
    elif kind == "fsdp":
        from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp

        mesh = Mesh({"data": D.world_size()})
        st = init_fsdp(Classifier(dropout_rate=0.0, num_layers=num_layers), sgd(1.0), 69, "cpu", mesh, "data", 16)
        tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data", gather_once=gather_once, scatter_once=gather_once))
        before = _clone(tr.full_params())
        tr.step(shard_batch(batch_full, mesh, "data"))
        after = _clone(tr.full_params())
    elif kind == "pp":
        from pipeline_parallel import build_mlp_pipeline

        mesh = Mesh({"data": dp, "pipe": D.world_size() // dp})
        tr = build_mlp_pipeline(cfg, mesh, "cpu", n_hidden_layers=n_hidden, dropout_rate=0.0,
                                num_microbatches=n_mb, tx=sgd(1.0))
        before = _clone(tr.state.params.state_dict())
        tr.step(shard_batch(batch_full, mesh, "data"))
        after = _clone(tr.state.params.state_dict())
    elif kind == "pp_lm":
        from jax_distributed_tuts_amd.models.transformer import TransformerConfig
        from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline, lm_batch

        lm_cfg = TransformerConfig(**LM_PROBE_CFG)
        mesh = Mesh({"data": dp, "pipe": D.world_size() // dp})
        tr, _ = build_lm_pipeline(mesh, "cpu", lm_cfg, num_microbatches=n_mb, tx=sgd(1.0))
        before = _clone(tr.state.params.state_dict())
        tr.step(shard_batch(lm_batch(lm_cfg, global_batch=2 * n_mb * dp, seed=5), mesh, "data"))
        after = _clone(tr.state.params.state_dict())
    else:
        raise ValueError(kind)
    _save(out_dir, f"probe_{kind}", {"before": before, "after": after})


def replication_desync(out_dir):
    """--check-replication on a DP trainer whose rank 1 was deliberately perturbed."""
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp, shard_batch
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.debug import ReplicationError, check_trainer_replication
    from jax_distributed_tuts_amd.utils.train_state import adamw

    mesh = Mesh({"data": D.world_size()})
    st = init_dp(Classifier(), adamw(1e-3), 69, "cpu", mesh)
    tr = DataParallelTrainer(st, mesh, DPConfig(4, "fused"))
    b = shard_batch(synthetic_batch(dp_config(), 70), mesh, "data")
    tr.step(b)
    check_trainer_replication(tr)  # healthy: passes
    if D.rank() == 1:
        st.params.p("output_dense/bias")[3] += 1e-6
    tr.step(b)
    try:
        check_trainer_replication(tr)
        res = "no-error"
    except ReplicationError as e:
        res = str(e)
    _save(out_dir, "repdesync", {"res": res})


def selftest_verdict(out_dir):
    """The xGMI / P2P self-test verdicts are collective: a failure seen by rank 1
    alone stops every rank at the same check, and a following collective still
    pairs up (a rank that returned alone would have paired its ``_agree`` with the
    others' next RCCL call)."""
    import torch.distributed as dist

    from jax_distributed_tuts_amd.comm.xgmi import XgmiComm

    c = object.__new__(XgmiComm)  # no device buffers: only the verdict plumbing
    c.group, c.rank, c.world, c.device = dist.group.WORLD, D.rank(), D.world_size(), torch.device("cpu")
    c.ctx = None
    c.error = lambda: 0
    c._fail = lambda what: False
    seen = []
    for it in range(4):
        ok = c._check(D.rank() == 1 and it == 2, f"check {it}")
        seen.append(ok)
        if not ok:
            break
    t = torch.tensor([float(len(seen))])
    dist.all_reduce(t)  # pairs up only if every rank stopped at the same check
    _save(out_dir, "verdict", {"seen": seen, "total": float(t.item())})


def unit_groups(out_dir):
    """A 1-rank gloo job whose 1-member data axis is a real process group
    (Mesh(unit_groups=True)): DP and FSDP issue their collectives exactly as at N > 1
    and must train exactly like the plain N = 1 step (CPU: bitwise)."""
    import torch.distributed as dist

    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import adamw

    dist.init_process_group("gloo", init_method="env://", rank=0, world_size=1)
    res = {}
    try:
        b = synthetic_batch(dp_config(), 70)
        for unit in (False, True):
            mesh = Mesh({"data": 1}, unit_groups=unit)
            res[f"active_{unit}"] = C.active(mesh, "data")
            st = init_dp(Classifier(dropout_rate=0.0), adamw(1e-3), 69, "cpu", mesh)
            tr = DataParallelTrainer(st, mesh, DPConfig(4, "loop"))
            res[f"dp_coll_{unit}"] = tr._coll
            for _ in range(3):
                tr.step(b)
            res[f"dp_{unit}"] = st.params.master.clone()
            st = init_fsdp(Classifier(num_layers=4, dropout_rate=0.0), adamw(1e-3), 69, "cpu", mesh, "data", 16)
            tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data"))
            res[f"fsdp_n1_{unit}"] = tr._n1
            for _ in range(3):
                tr.step(b)
            res[f"fsdp_{unit}"] = st.params.master.clone()
    finally:
        dist.destroy_process_group()
    _save(out_dir, "unit", res)
