"""RCCL collectives recorded inside the step's hipGraph (the fallback transport when
the xGMI kernels are unavailable or measured slower).

A 1-rank nccl process group on the box's one GPU plus ``Mesh(unit_groups=True)``
makes the trainers issue exactly the RCCL calls of an N-GPU job (all-reduce,
all-gather, reduce-scatter) on a 1-member data axis.  The captured step -- the
collective inside the graph, as the reference's whole step sits under one ``jit``
(data_paral.py:241-251, param_sharding.py:370-379) -- must replay to the same
parameters as the eager step."""
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_world1():
    from jax_distributed_tuts_amd.runtime import dist as D
    from jax_distributed_tuts_amd.runtime.launch import free_port

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0, world_size=1,
                            device_id=dev)
    D._STATE["device"] = dev
    try:
        yield dev
    finally:
        dist.destroy_process_group()
        D._STATE["device"] = None


def _close(got, want, steps: int):
    """Captured vs eager parameters after ``steps`` AdamW steps: the same kernels up to
    fp32 summation order (atomics), so at most ~lr per step apart anywhere and almost
    everywhere equal."""
    d = (got - want).abs()
    assert float(d.max()) <= 2 * 1e-3 * steps + 1e-6
    assert float((d > 5e-5).float().mean()) < 5e-3


def _batch(dev):
    from data_paral import synthetic_batch
    from jax_distributed_tuts_amd.utils.config import dp_config
    from jax_distributed_tuts_amd.utils.train_state import Batch

    b = synthetic_batch(dp_config(), 70)
    return Batch(b.inputs.to(dev), b.labels.to(dev))


def test_raw_rccl_collectives_replay_from_a_graph(nccl_world1):
    from jax_distributed_tuts_amd.comm import collectives as C
    from jax_distributed_tuts_amd.runtime.dist import Mesh, collectives_capturable

    dev = nccl_world1
    mesh = Mesh({"data": 1}, unit_groups=True)
    assert C.active(mesh, "data") and collectives_capturable()
    x = torch.arange(4096, device=dev, dtype=torch.float32)
    full = torch.empty(4096, device=dev)
    part = torch.empty(4096, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        C.psum_(x, mesh, "data")
        x.mul_(2.0)
        C.all_gather(x, mesh, "data", out=full)
        C.psum_scatter(full, mesh, "data", out=part)
    for k in range(3):
        x.copy_(torch.arange(4096, device=dev, dtype=torch.float32) + k)
        g.replay()
        torch.cuda.synchronize()
        want = (torch.arange(4096, device=dev, dtype=torch.float32) + k) * 2
        assert torch.equal(x, want) and torch.equal(full, want) and torch.equal(part, want)


@pytest.mark.parametrize("accum", ["kernel", "loop"])
def test_dp_step_graph_holds_the_rccl_allreduce(nccl_world1, accum):
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.train_state import adamw

    dev = nccl_world1
    mesh = Mesh({"data": 1}, unit_groups=True)
    b = _batch(dev)
    runs = []
    for captured in (False, True):
        st = init_dp(Classifier(dropout_rate=0.0), adamw(1e-3), 69, dev, mesh)
        tr = DataParallelTrainer(st, mesh, DPConfig(4, accum, comm="rccl"))
        assert tr._coll and tr.xg is None and tr.comm_backend == "rccl"
        tr.step(b)
        if captured:
            tr.capture(b, steps_per_graph=2)
            assert tr.graph[0] == "one", "the RCCL all-reduce must sit inside the step graph"
            assert tr.multi is not None and tr.multi[0] == 2
            tr.run_steps(b, 4)
        else:
            for _ in range(4):
                tr.step(b)
        torch.cuda.synchronize()
        tr.finalize()
        runs.append((st.params.master.clone(), tr.metrics.clone(), int(st.opt_state["count"].item())))
    (pe, me, ce), (pc, mc, cc) = runs
    assert ce == cc == 5
    _close(pc, pe, 5)
    torch.testing.assert_close(mc, me, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("num_layers,fused", [(2, True), (4, True), (2, False)])
def test_fsdp_step_graph_holds_the_rccl_collectives(nccl_world1, num_layers, fused):
    from jax_distributed_tuts_amd.models.mlp import Classifier
    from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
    from jax_distributed_tuts_amd.runtime.dist import Mesh
    from jax_distributed_tuts_amd.utils.train_state import adamw

    dev = nccl_world1
    mesh = Mesh({"data": 1}, unit_groups=True)
    b = _batch(dev)
    runs = []
    for captured in (False, True):
        st = init_fsdp(Classifier(num_layers=num_layers, dropout_rate=0.0), adamw(1e-3), 69, dev, mesh, "data", 16)
        tr = FSDPTrainer(st, mesh, FSDPConfig(4, 16, "data", gather_once=True, scatter_once=True,
                                              fused_kernels=fused, comm="rccl"))
        assert not tr._n1 and tr.sp.xg is None and tr.comm_backend == "rccl" and tr.capturable
        tr.step(b)
        if captured:
            assert tr.capture(b, steps_per_graph=2)
            tr.run_steps(b, 4)
        else:
            for _ in range(4):
                tr.step(b)
        torch.cuda.synchronize()
        tr.finalize()
        runs.append((st.params.master.clone(), tr.metrics.clone()))
    (pe, me), (pc, mc) = runs
    _close(pc, pe, 5)
    torch.testing.assert_close(mc, me, rtol=1e-3, atol=1e-3)
